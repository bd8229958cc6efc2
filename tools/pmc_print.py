"""Average rocprofv3 counter values per kernel: python tools/pmc_print.py <counter_collection.csv> [substr]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if sub in k:
        waves = sum(d["SQ_WAVES"]) / len(d["SQ_WAVES"]) if "SQ_WAVES" in d else None
        out = {c: f"{sum(v) / len(v):.4g}" for c, v in d.items()}
        if waves:
            out.update({f"{c}/wave": f"{sum(v) / len(v) / waves:.1f}" for c, v in d.items()
                        if c.startswith("SQ_INSTS")})
        print(k, out)
