"""Per-kernel mean of every counter in rocprofv3 --pmc CSVs (counter_collection.csv), for the
dispatches whose kernel name contains a substring, in dispatch order per grid size:
    python tools/pmc_kernels.py SUBSTRING run_counter_collection.csv [...]"""
import collections
import csv
import sys

sub = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[2:]:
    for r in csv.DictReader(open(path)):
        if sub not in r["Kernel_Name"]:
            continue
        key = (r["Kernel_Name"].split("(")[0][-40:], r["Grid_Size"])
        vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for key, cs in vals.items():
    print(key)
    for c, v in sorted(cs.items()):
        print(f"  {c:32s} n={len(v):3d} mean={sum(v) / len(v):.6g}")
