#!/bin/bash
# The x6 GEMM's raw-X ring depth (G6_NX_SLOTS: X of k-step j + NX - 1 loads during step j; 6
# shipped, 7 = 160 KB of LDS with the W ring): time per call on the shortcut shapes.
#   tools/build_variant.sh nx7 "-DG6_NX_SLOTS=7"; ... nx5; tools/x6_ring_ab.sh -> gpurun_out/x6ring/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/x6ring; mkdir -p $O
for v in default nx7 nx5 default nx7 nx5; do
  if [ $v = default ]; then lib=""; else lib=$R/samplers_amd/lib/variants/lib_$v.so; fi
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 200 python3 -u $R/tools/bench_gemm_x6.py > $O/gemm_$v.jsonl 2>&1 || exit $?
  echo "== $v"; grep -h "x6" $O/gemm_$v.jsonl | cut -c1-130 | head -3
done
SAMPLERS_HIP_LIB=$R/samplers_amd/lib/variants/lib_nx7.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  $R/tests/test_gemm_x6_gpu.py > $O/nx7_tests.log 2>&1; tail -1 $O/nx7_tests.log
