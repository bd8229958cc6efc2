"""Per-dispatch rocprofv3 counter values for kernels matching a substring:
python tools/pmc_disp.py <dir with pmc_*/ *counter_collection.csv> <substr> [exclude]"""
import collections
import csv
import glob
import sys

d = collections.defaultdict(dict)
sub = sys.argv[2]
excl = sys.argv[3] if len(sys.argv) > 3 else None
for path in sorted(glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if sub not in k or (excl and excl in k):
            continue
        key = (path.split("/")[-2], int(r["Dispatch_Id"]))
        d[key][r["Counter_Name"]] = d[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        d[key]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for key in sorted(d):
    print(key, {a: f"{b:.4g}" for a, b in sorted(d[key].items())})
