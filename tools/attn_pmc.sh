#!/bin/bash
# SQ counters of the attention forward kernels (tools/bench_attention.py MODE), one rocprofv3
# --pmc pass per counter set:  MODE=x6 tools/attn_pmc.sh -> gpurun_out/attn_pmc/<MODE>/p*/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/attn_pmc/${MODE:-x6}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
while read -r set; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python3 $R/tools/bench_attention.py ${MODE:-x6} > $O/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done <<SETS
SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU
SETS
python3 - "$O" <<'PY'
import csv, glob, sys, collections
out = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "attn" in r["Kernel_Name"]:
            k = r["Kernel_Name"].split("(")[0][-40:]
            out[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in out.items():
    print(k, {c: round(sum(v) / len(v), 1) for c, v in sorted(d.items())})
PY
