# pipelined direct bf16x6 conv: tests, then bench (default = pipelined, variant = previous loop)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_x6d_gpu.py > gpurun_out/x6d_tests.log 2>&1
timeout -k 10 200 python -u tools/bench_conv_x6.py > gpurun_out/c6pipe.jsonl 2>&1
SAMPLERS_HIP_LIB=samplers_amd/lib/variants/lib_c6_nopipe.so timeout -k 10 200 python -u tools/bench_conv_x6.py > gpurun_out/c6nopipe.jsonl 2>&1
