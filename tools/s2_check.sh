#!/bin/bash
set -o pipefail
O=gpurun_out/s2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_conv_gpu.py tests/test_latent_full_gpu.py -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_psld.py > $O/psld.log 2>&1 || exit $?
tail -1 $O/psld.log | cut -c1-300
timeout -k 10 400 python -u tools/bench_resample.py > $O/resample.log 2>&1 || exit $?
tail -1 $O/resample.log | cut -c1-300
