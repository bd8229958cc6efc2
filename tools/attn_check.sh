#!/bin/bash
set -o pipefail
O=gpurun_out/att; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -15 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_attention.py > $O/attn_fused.log 2>&1 || exit $?
grep -v amdgpu $O/attn_fused.log
timeout -k 10 900 python -u -m pytest tests/test_latent_full_gpu.py -x -q --timeout 400 --timeout-method thread > $O/latent_tests.log 2>&1; rc=$?; tail -2 $O/latent_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_psld.py > $O/psld.log 2>&1 || exit $?
tail -1 $O/psld.log | cut -c1-250
timeout -k 10 400 python -u tools/bench_resample.py > $O/resample.log 2>&1 || exit $?
tail -1 $O/resample.log | cut -c1-250
