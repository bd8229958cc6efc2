#!/bin/bash
# Correctness + isolated timing of the DPS passes (inpaint; pass 2 re-reading v: REUSE_V=1, or
# re-deriving it from y: REUSE_V=0) per library variant (samplers_amd/lib/variants/lib_dps_*.so).
set -o pipefail
O=gpurun_out/dpsv; mkdir -p $O
for v in default ${VARIANTS}; do
  if [ $v = default ]; then lib=""; else lib=samplers_amd/lib/variants/lib_dps_$v.so; fi
  if [ -n "$TESTS" ]; then
    env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py tests/test_dps_gpu.py tests/test_full_size_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test_$v.log 2>&1 || { echo "$v: tests failed"; tail -20 $O/test_$v.log; exit 1; }
    echo "$v: $(tail -1 $O/test_$v.log)"
  fi
  for rv in 0 1; do
    env ${lib:+SAMPLERS_HIP_LIB=$lib} OPS=inpaint REUSE_V=$rv timeout -k 10 120 python -u tools/bench_kernels.py $v > $O/bench_${v}_rv$rv.jsonl 2>&1 || exit $?
    grep -h "dps_" $O/bench_${v}_rv$rv.jsonl | sed "s/^/rv$rv /"
  done
done
