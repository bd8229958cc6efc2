#!/bin/bash
# SQ / cache counters of the Winograd tile on two layer shapes (tools/bench_conv.py, forward
# only), one rocprofv3 --pmc pass per counter set (MI355X_MICROARCH.md: per-pass slot limits).
#   LIB=samplers_amd/lib/variants/lib_x.so TAG=x tools/wino_pmc.sh -> gpurun_out/wino_pmc/<TAG>/p*/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/wino_pmc/${TAG:-default}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export CUSTOM=${CUSTOM:-"64,128,128,256,256;64,512,256,64,64"} ROWS=${ROWS:-wino_fwd}
[ -n "$LIB" ] && export SAMPLERS_HIP_LIB=$R/$LIB
i=0
while read -r set; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python3 $R/tools/bench_conv.py > $O/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done <<SETS
SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU
TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum
SETS
echo "pmc ${TAG:-default} done"
