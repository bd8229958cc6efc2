#!/bin/bash
# Blur streaming-pass variants (samplers_amd/lib/variants/lib_blur_*.so) in the blur step.
set -o pipefail
O=gpurun_out/blur; mkdir -p $O
for v in default ${VARIANTS}; do
  if [ $v = default ]; then lib=""; else lib=samplers_amd/lib/variants/lib_blur_$v.so; fi
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 120 python -u -m pytest tests/test_full_size_gpu.py -k blur -x -q --timeout 100 --timeout-method thread > $O/test_$v.log 2>&1 || { tail -5 $O/test_$v.log; exit 1; }
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 200 python -u bench.py --config blur --no-cpu-baseline --steps 5 > $O/bench_$v.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('$O/bench_$v.log').read().strip().splitlines()[-1]); g=d['guidance_kernels']; print('$v', d['value'], g['dps_residual'], d['guidance_roofline']['frac'])"
done
