"""Per-dispatch counters of one kernel from rocprofv3 --pmc passes (each pass a separate run of
the same program: dispatch k of the kernel in one pass is dispatch k in the others).  Values
summed over the CSV's rows of a dispatch (per-XCD / per-SE rows), then grouped into blocks
of --per consecutive dispatches (one block per problem shape of the program):
    python tools/pmc_dispatch.py SUBSTRING --per 7 p1/run_counter_collection.csv p2/... """
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument("sub")
ap.add_argument("csvs", nargs="+")
ap.add_argument("--per", type=int, default=0)
a = ap.parse_args()
blocks = collections.defaultdict(lambda: collections.defaultdict(list))
for path in a.csvs:
    disp = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if a.sub not in r["Kernel_Name"]:
            continue
        d = disp.setdefault(r["Dispatch_Id"], {"_ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for k, d in enumerate(disp.values()):
        b = k // a.per if a.per else 0
        for c, v in d.items():
            blocks[b][c].append(v)
for b, cs in sorted(blocks.items()):
    m = {c: sum(v[1:]) / max(1, len(v) - 1) if len(v) > 2 else sum(v) / len(v) for c, v in cs.items()}
    print(f"block {b}: {len(cs['_ns'])} dispatches, mean {m['_ns'] / 1e6:.3f} ms (first dispatch of a block excluded)")
    for c, v in sorted(m.items()):
        print(f"  {c:32s} {v:.6g}")
    if "GRBM_GUI_ACTIVE" in m:
        clk = m["GRBM_GUI_ACTIVE"] / 8 / (m["_ns"] * 1e-9) / 1e9
        print(f"  -> clock {clk:.3f} GHz (GRBM_GUI_ACTIVE / 8 XCDs / time)")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            print(f"  -> MFMA busy {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] / 8 * 256 * 4):.3f} "
                  "of SIMD cycles (256 CUs x 4 SIMDs)")
    if "SQ_WAVE_CYCLES" in m:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in m:
                print(f"  -> {c} / SQ_WAVE_CYCLES {m[c] / m['SQ_WAVE_CYCLES']:.3f}")
    if "SQ_LDS_IDX_ACTIVE" in m and m["SQ_LDS_IDX_ACTIVE"]:
        print(f"  -> LDS bank conflict / LDS active {m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:.3f}")
