#!/bin/bash
# PMC passes (one rocprofv3 run each) over tools/bench_kernels.py OPS=blur for the libs named
# on the command line (build/variants/lib_blur_<name>.so).  Output: gpurun_out/pmc_blur/<lib>/<pass>/
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
P3="FETCH_SIZE"
P4="TCC_HIT_sum TCC_MISS_sum"
for lib in "$@"; do
  i=0
  for p in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i+1))
    SAMPLERS_HIP_LIB=$R/build/variants/lib_blur_$lib.so OPS=blur timeout -s KILL 90 rocprofv3 --pmc $p \
      --output-format csv -d $R/gpurun_out/pmc_blur/$lib/p$i -o run -- python3 $R/tools/bench_kernels.py $lib \
      > $R/gpurun_out/pmc_blur/$lib.p$i.log 2>&1 || exit 1
  done
done
