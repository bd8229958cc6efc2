# direct bf16x6 conv: GPU tests, then the DPS step A/B (default tiles vs SAMPLERS_AMD_CONV=x6d)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_x6d_gpu.py > gpurun_out/x6d_tests.log 2>&1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_auto.json 2> gpurun_out/ab_auto.err
SAMPLERS_AMD_CONV=x6d timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_x6d.json 2> gpurun_out/ab_x6d.err
