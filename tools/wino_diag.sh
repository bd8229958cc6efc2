#!/bin/bash
# Winograd tile diagnostics (tools/build_variant.sh NAME "-DSP_WINO_EXP=6" ...) against the default
# library on layers of one output geometry and several input-channel counts (time = a + b * cin:
# a = the per-tile fixed cost, b = the k-steps):  VARIANTS="wx6" tools/wino_diag.sh -> gpurun_out/winodiag/
set -o pipefail
O=gpurun_out/winodiag; mkdir -p $O
SH=${CUSTOM:-"64,128,128,256,256;64,256,128,256,256;64,384,128,256,256;64,128,256,128,128;64,256,256,128,128;64,512,256,128,128"}
for v in default ${VARIANTS}; do
  if [ $v = default ]; then lib=""; else lib=samplers_amd/lib/variants/lib_$v.so; fi
  env ${lib:+SAMPLERS_HIP_LIB=$lib} CUSTOM="$SH" ROWS=wino_fwd,wino_bwd_input timeout -k 10 200 python -u tools/bench_conv.py > $O/conv_$v.jsonl 2>&1 || exit $?
  echo "== $v"; grep -h wino $O/conv_$v.jsonl | cut -c1-110
done
