#!/bin/bash
# Winograd tile variants (samplers_amd/lib/variants/lib_wino_*.so, tools/build_variant.sh) in the
# headline step, after the conv tests on the default library:
#   VARIANTS="32 44" tools/wino_ab.sh   ->  gpurun_out/wino/{tests.log,bench_*.log}
set -o pipefail
O=gpurun_out/wino; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for v in default ${VARIANTS}; do
  if [ $v = default ]; then lib=""; else lib=samplers_amd/lib/variants/lib_wino_$v.so; fi
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps ${STEPS:-5} > $O/bench_$v.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('$O/bench_$v.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'])"
done
