#!/bin/bash
# GroupNorm kernels: GPU tests that exercise them, tools/bench_gn.py, and the headline step.
set -o pipefail
O=gpurun_out/gn; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_groupnorm_gpu.py tests/test_latent_full_gpu.py tests/test_dps_gpu.py -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_gn.py > $O/gn_default.log 2>&1 || exit $?
grep -v amdgpu.ids $O/gn_default.log | cut -c1-160
timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-250
