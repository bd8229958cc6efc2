#!/bin/bash
# The bf16 MFMA shape lever on the token-major linears (G6_EXP=7, timing only): tools/build_variant.sh e7 "-DG6_EXP=7"; tools/x6_linear_shape_ab.sh
set -o pipefail
mkdir -p gpurun_out/linab
for v in default e7 default e7; do
  if [ $v = default ]; then lib=""; else lib=samplers_amd/lib/variants/lib_$v.so; fi
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 200 python -u tools/bench_linear_x6.py > gpurun_out/linab/lin_$v.jsonl 2>&1 || exit $?
  echo "== $v"; grep -h "tokens" gpurun_out/linab/lin_$v.jsonl | cut -c1-150
done
