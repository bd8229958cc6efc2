#!/bin/bash
# bf16 ResnetBlock A/B: GN2's moments from conv1's epilogue (default) vs conv1 + two-pass GroupNorm
set -o pipefail
mkdir -p gpurun_out/fs
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bf16_gpu.py -k "resnet or celebahq" > gpurun_out/fs/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --dtype bf16 --no-cpu-baseline > gpurun_out/fs/bench_on.json 2> gpurun_out/fs/bench_on.log || exit $?
SAMPLERS_AMD_BF16_GNFWD=0 timeout -k 10 300 python -u bench.py --dtype bf16 --no-cpu-baseline > gpurun_out/fs/bench_off.json 2> gpurun_out/fs/bench_off.log
