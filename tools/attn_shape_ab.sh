#!/bin/bash
# The clock lever of the bf16 MFMA shape inside the split-bf16 attention forward: the shipped
# kernel against A6_EXP=7 (each v_mfma_f32_32x32x16_bf16 replaced by two 16x16x32 ones on the same
# operands: the same MACs, wrong results) — time and the held clock / MFMA busy (tools/sq_pmc.sh).
#   tools/build_variant.sh a7 "-DA6_EXP=7"; tools/attn_shape_ab.sh  ->  gpurun_out/attnshape/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/attnshape; mkdir -p $O
for v in default a7; do
  if [ $v = default ]; then lib=""; else lib=$R/samplers_amd/lib/variants/lib_$v.so; fi
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 200 python3 -u $R/tools/bench_attention.py x6 > $O/attn_$v.jsonl 2>&1 || exit $?
  env ${lib:+SAMPLERS_HIP_LIB=$lib} FILTER=k_attn6 NAME=attn_$v timeout -k 10 400 bash $R/tools/sq_pmc.sh tools/bench_attention.py x6 > $O/sq_$v.txt 2>&1 || exit $?
  echo "== $v"; grep -h "fwd_ms" $O/attn_$v.jsonl | cut -c1-160; grep -h "k_attn6" $O/sq_$v.txt | cut -c1-160
done
