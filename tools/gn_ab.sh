#!/bin/bash
# GroupNorm variants on the UNet's shapes (tools/bench_gn.py) and in the headline step.
set -o pipefail
O=gpurun_out/gn; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_groupnorm_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_gn.py > $O/gn_default.log 2>&1 || exit $?
for v in ${VARIANTS:-team}; do
  SAMPLERS_HIP_LIB=samplers_amd/lib/variants/lib_gn_$v.so timeout -k 10 200 python -u tools/bench_gn.py > $O/gn_$v.log 2>&1 || exit $?
done
for f in $O/gn_*.log; do echo "== $f"; grep -v amdgpu.ids $f | cut -c1-160; done
