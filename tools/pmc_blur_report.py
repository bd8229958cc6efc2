"""Summarise gpurun_out/pmc_blur/<lib>/p*/run_counter_collection.csv for the blur DPS pass
(kernel names containing k_blur): mean per dispatch."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_blur"
for lib in sorted(glob.glob(f"{root}/*/")):
    vals = collections.defaultdict(list)
    ns = []
    for path in sorted(glob.glob(f"{lib}/p*/run_counter_collection.csv")):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(path)):
            if "k_blur" not in r["Kernel_Name"]:
                continue
            per[(int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
        for (d, cname), v in per.items():
            vals[cname].append(v)
    m = {k: sum(v) / len(v) for k, v in vals.items()}
    w = m.get("SQ_WAVES", 1)
    out = {k: round(v, 1) for k, v in sorted(m.items())}
    print(lib.split("/")[-2], out)
    if "SQ_WAVE_CYCLES" in m:
        print("   per wave: VALU %.0f LDS %.0f VMEM %.0f SALU %.0f | wave-cycles %.0f (x4) busy %.0f" % (
            m.get("SQ_INSTS_VALU", 0) / w, m.get("SQ_INSTS_LDS", 0) / w, m.get("SQ_INSTS_VMEM", 0) / w,
            m.get("SQ_INSTS_SALU", 0) / w, m["SQ_WAVE_CYCLES"] / w * 4, m.get("SQ_BUSY_CYCLES", 0)))
    if "FETCH_SIZE" in m:
        print("   HBM fetch (x2 gfx950) %.1f MB; TCC hit %.3f" % (
            2 * m["FETCH_SIZE"] * 1024 / 1e6,
            m.get("TCC_HIT_sum", 0) / max(1, m.get("TCC_HIT_sum", 0) + m.get("TCC_MISS_sum", 0))))
