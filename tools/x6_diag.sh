#!/bin/bash
# bf16x6 GEMM variants (tools/build_variant.sh NAME "-DG6_EXP=5" ...) against the default library
# on the linear (tools/bench_linear_x6.py) and shortcut (tools/bench_gemm_x6.py) shapes:
#   VARIANTS="x6e5" tools/x6_diag.sh  ->  gpurun_out/x6diag/
set -o pipefail
O=gpurun_out/x6diag; mkdir -p $O
for v in default ${VARIANTS}; do
  if [ $v = default ]; then lib=""; else lib=samplers_amd/lib/variants/lib_$v.so; fi
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 200 python -u tools/bench_linear_x6.py > $O/linear_$v.jsonl 2>&1 || exit $?
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 200 python -u tools/bench_gemm_x6.py > $O/gemm_$v.jsonl 2>&1 || exit $?
  echo "== $v"; grep -h "tokens" $O/linear_$v.jsonl | cut -c1-110 | head -4; grep -h "x6" $O/gemm_$v.jsonl | cut -c1-160 | head -3
done
