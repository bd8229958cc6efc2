#!/bin/bash
# What the x6 GEMM's per-k-step workgroup barrier costs: the shipped tile against G6_EXP=8 (no
# barrier in the k loop: wrong results, timing only) and G6_EXP=6 (MFMAs only).
#   tools/build_variant.sh e8 "-DG6_EXP=8"; tools/x6_barrier_ab.sh  ->  gpurun_out/x6barrier/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/x6barrier; mkdir -p $O
for v in default e8 default e8; do
  if [ $v = default ]; then lib=""; else lib=$R/samplers_amd/lib/variants/lib_$v.so; fi
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 200 python3 -u $R/tools/bench_gemm_x6.py > $O/gemm_$v.jsonl 2>&1 || exit $?
  echo "== $v"; grep -h "x6" $O/gemm_$v.jsonl | cut -c1-130 | head -4
done
