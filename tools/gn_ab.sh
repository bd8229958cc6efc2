#!/bin/bash
# GroupNorm cache-policy variants (samplers_amd/lib/variants/lib_gn_*.so) in tools/bench_gn.py and
# the headline step, after the GroupNorm parity tests.  Output: gpurun_out/gnab/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/gnab
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_groupnorm_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for v in default ${VARIANTS}; do
  if [ $v = default ]; then lib=""; else lib=$R/samplers_amd/lib/variants/lib_gn_$v.so; fi
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 200 python -u tools/bench_gn.py > $O/gn_$v.log 2>&1 || exit $?
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 5 > $O/bench_$v.log 2>&1 || exit $?
  echo "== $v"; grep '"shape"' $O/gn_$v.log | head -4
  python -c "import json; d=json.loads(open('$O/bench_$v.log').read().strip().splitlines()[-1]); print('$v bench', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
