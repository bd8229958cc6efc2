"""Per-dispatch means of the SQ counters tools/g6_pmc.sh collected for k_gemm_x6<false, false>,
with the derived ratios (wave-cycle shares, MFMA busy share, LDS bank-conflict share).
    python tools/g6_pmc_summary.py gpurun_out/g6pmc default old ..."""
import collections
import csv
import glob
import json
import sys


def main():
    root, names = sys.argv[1], sys.argv[2:]
    for v in names:
        agg, n = collections.defaultdict(float), collections.Counter()
        for f in glob.glob(f"{root}/{v}/p*/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "k_gemm_x6<false, false>" not in r["Kernel_Name"]:
                    continue
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
                n[r["Counter_Name"]] += 1
        d = {k: x / n[k] for k, x in agg.items()}
        if "SQ_WAVE_CYCLES" not in d or "GRBM_GUI_ACTIVE" not in d:
            files = glob.glob(f"{root}/{v}/**", recursive=True)
            kernels = set()
            for f in files:
                if f.endswith("counter_collection.csv"):
                    kernels |= {r["Kernel_Name"][:60] for r in csv.DictReader(open(f))}
            print(json.dumps({"lib": v, "missing": sorted(d), "files": files[:12], "kernels": sorted(kernels)[:20]}))
            continue
        w = d["SQ_WAVE_CYCLES"]
        out = {"lib": v, "dispatches": n["SQ_WAVES"], "means": {k: round(x) for k, x in sorted(d.items())},
               "wait_any_per_wave_cycle": round(d["SQ_WAIT_ANY"] / w, 3),
               "wait_inst_any_per_wave_cycle": round(d["SQ_WAIT_INST_ANY"] / w, 3),
               "active_inst_per_wave_cycle": round(d["SQ_ACTIVE_INST_ANY"] / w, 3),
               "wait_inst_lds_per_wave_cycle": round(d["SQ_WAIT_INST_LDS"] / w, 3),
               "mfma_busy_share": round(d["SQ_VALU_MFMA_BUSY_CYCLES"] / (d["GRBM_GUI_ACTIVE"] * 1024), 3),
               "lds_bank_conflict_share": round(d["SQ_LDS_BANK_CONFLICT"] / max(d["SQ_LDS_IDX_ACTIVE"], 1), 3),
               "valu_insts_per_wave": round(d["SQ_INSTS_VALU"] / d["SQ_WAVES"]),
               "lds_insts_per_wave": round(d["SQ_INSTS_LDS"] / d["SQ_WAVES"])}
        print(json.dumps(out))


if __name__ == "__main__":
    main()
