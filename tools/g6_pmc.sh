#!/bin/bash
# SQ counters of the bf16x6 GEMM (tools/bench_gemm_x6.py, case 0: 64x(128+128)->128 at 256^2) for
# the default library and the variants named in G6_LIST, two rocprofv3 passes each (counter
# limits per pass).  Output: gpurun_out/g6pmc/<lib>/p<k>/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g6pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
for v in default ${G6_LIST}; do
  if [ $v = default ]; then lib=$R/samplers_amd/lib/libsamplers_hip.so; else lib=$R/samplers_amd/lib/variants/lib_g6_$v.so; fi
  k=0
  for P in "$P1" "$P2"; do
    k=$((k+1))
    SAMPLERS_HIP_LIB=$lib G6_CASES=0 timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/$v/p$k -o run -- \
      python3 $R/tools/bench_gemm_x6.py > $O/$v.p$k.log 2>&1 || { echo "$v pass $k failed"; tail -5 $O/$v.p$k.log; exit 1; }
  done
  echo "== $v done"
done
python3 $R/tools/g6_pmc_summary.py $O default ${G6_LIST} > $O/summary.jsonl && cat $O/summary.jsonl
rm -rf $O/default $(for v in ${G6_LIST}; do echo $O/$v; done)
