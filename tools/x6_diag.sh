set -o pipefail
O=gpurun_out/x6diag; mkdir -p $O
for v in default x6old x6e5; do
  if [ $v = default ]; then lib=""; else lib=samplers_amd/lib/variants/lib_$v.so; fi
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 200 python -u tools/bench_linear_x6.py > $O/linear_$v.jsonl 2>&1 || exit $?
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 200 python -u tools/bench_gemm_x6.py > $O/gemm_$v.jsonl 2>&1 || exit $?
  echo "== $v"; grep -h "tokens\|x6" $O/linear_$v.jsonl | cut -c1-110 | head -4; grep -h "x6" $O/gemm_$v.jsonl | cut -c1-160 | head -3
done
