#!/bin/bash
# GroupNorm variants (tools/build_variant.sh NAME ...) against the default library: the GroupNorm
# tests, tools/bench_gn.py and the headline bench.   VARIANTS="gnold" tools/gn_ab.sh -> gpurun_out/gn/
set -o pipefail
O=gpurun_out/gn; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_groupnorm_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for v in default ${VARIANTS}; do
  if [ $v = default ]; then lib=""; else lib=samplers_amd/lib/variants/lib_$v.so; fi
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 200 python -u tools/bench_gn.py > $O/gn_$v.jsonl 2>&1 || exit $?
  echo "== $v"; grep '"single_pass": 1' $O/gn_$v.jsonl | cut -c1-120
done
for v in ${BENCH_VARIANTS}; do
  if [ $v = default ]; then lib=""; else lib=samplers_amd/lib/variants/lib_$v.so; fi
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 5 > $O/bench_$v.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('$O/bench_$v.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
