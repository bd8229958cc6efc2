#!/bin/bash
# The clock lever of the bf16 MFMA shape inside the x6 GEMM: the shipped tile against G6_EXP=7
# (every v_mfma_f32_32x32x16_bf16 replaced by two 16x16x32 ones on the same operands: the same
# MACs, wrong results) — time per call and the held clock / MFMA busy (tools/sq_pmc.sh).
#   tools/build_variant.sh e7 "-DG6_EXP=7"; tools/x6_shape_ab.sh  ->  gpurun_out/x6shape/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/x6shape; mkdir -p $O
for v in default e7; do
  if [ $v = default ]; then lib=""; else lib=$R/samplers_amd/lib/variants/lib_$v.so; fi
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 200 python3 -u $R/tools/bench_gemm_x6.py > $O/gemm_$v.jsonl 2>&1 || exit $?
  env ${lib:+SAMPLERS_HIP_LIB=$lib} G6_CASES=0 FILTER=k_gemm_x6 NAME=x6_$v timeout -k 10 400 bash $R/tools/sq_pmc.sh tools/bench_gemm_x6.py > $O/sq_$v.txt 2>&1 || exit $?
  echo "== $v"; grep -h "x6" $O/gemm_$v.jsonl | cut -c1-120 | head -4; grep -h "k_gemm_x6" $O/sq_$v.txt | cut -c1-160
done
