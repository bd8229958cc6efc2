#!/bin/bash
# SQ counters (and the clock the chip holds: GRBM_GUI_ACTIVE per XCD over the dispatch) of the
# kernels whose names contain FILTER, under any python command, one rocprofv3 --pmc pass per
# counter set:   FILTER=k_gemm_x6 NAME=x6 tools/sq_pmc.sh tools/bench_gemm_x6.py [args]
#                -> gpurun_out/sq_pmc/<NAME>/p*/ and a per-kernel summary on stdout
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sq_pmc/${NAME:-run}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
while read -r set; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/p$i -o run -- python3 $R/"$@" > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/p$i.log; exit 1; }
done <<SETS
SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU
SETS
python3 - "$O" "${FILTER:-k_}" <<'PY'
import csv, glob, sys, collections
out = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p1/**/*counter_collection.csv", recursive=True) + \
         glob.glob(sys.argv[1] + "/p2/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if sys.argv[2] in r["Kernel_Name"]:
            k = r["Kernel_Name"].split("(")[0][-48:]
            out[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in glob.glob(sys.argv[1] + "/p1/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if sys.argv[2] in r["Kernel_Name"]:
            dur[r["Kernel_Name"].split("(")[0][-48:]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
for k, d in out.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    t = sum(dur[k]) / len(dur[k]) if dur.get(k) else None
    ghz = m.get("GRBM_GUI_ACTIVE", 0) / 8 / t / 1e9 if t else None
    busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / 1024 / (m.get("GRBM_GUI_ACTIVE", 1) / 8)
    print(k, {"mean_ms": round(t * 1e3, 4) if t else None, "clock_GHz": round(ghz, 2) if ghz else None,
              "mfma_busy": round(busy, 3), **{c: round(v, 1) for c, v in sorted(m.items())}})
PY
