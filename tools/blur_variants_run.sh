#!/bin/bash
# Correctness + isolated timing of the blur DPS pass for each library variant
# (samplers_amd/lib/variants/lib_blur_<name>.so, tools/build_blur_variants.sh).
#   VARIANTS="old pf1 ..." bash tools/blur_variants_run.sh      -> gpurun_out/blurv/
set -o pipefail
O=gpurun_out/blurv; mkdir -p $O
for v in default ${VARIANTS}; do
  if [ $v = default ]; then lib=""; else lib=samplers_amd/lib/variants/lib_blur_$v.so; fi
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 200 python -u -m pytest tests/test_hip_kernels.py tests/test_full_size_gpu.py -k blur -x -q --timeout 100 --timeout-method thread > $O/test_$v.log 2>&1 || { echo "$v: tests failed"; tail -20 $O/test_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/test_$v.log)"
  env ${lib:+SAMPLERS_HIP_LIB=$lib} OPS=blur timeout -k 10 120 python -u tools/bench_kernels.py $v > $O/bench_$v.jsonl 2>&1 || exit $?
  grep dps_residual $O/bench_$v.jsonl
done
