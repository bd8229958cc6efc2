#!/bin/bash
# bf16 ResnetBlock VJP: the 1x1 shortcut's input gradient as one GEMM over cat(x, skip) read by GN1's VJP as a
# combined addend (default) vs one GEMM per part (SAMPLERS_AMD_BF16_SCVJP=0); tests first
set -o pipefail
mkdir -p gpurun_out/scvjp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bf16_gpu.py -k "resnet or celebahq or groupnorm" > gpurun_out/scvjp/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --dtype bf16 --no-cpu-baseline > gpurun_out/scvjp/dps_on.json 2> gpurun_out/scvjp/dps_on.log || exit $?
SAMPLERS_AMD_BF16_SCVJP=0 timeout -k 10 300 python -u bench.py --dtype bf16 --no-cpu-baseline > gpurun_out/scvjp/dps_off.json 2> gpurun_out/scvjp/dps_off.log || exit $?
timeout -k 10 300 python -u bench.py --dtype bf16 --no-cpu-baseline > gpurun_out/scvjp/dps_on2.json 2> gpurun_out/scvjp/dps_on2.log
