set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_distributed_gpu.py tests/test_groupnorm_gpu.py > gpurun_out/r5/dist_tests.log 2>&1 && \
SAMPLERS_AMD_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --config blur --gpus 8 --batch 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r5/bench_gloo8_blur.json 2> gpurun_out/r5/bench_gloo8_blur.log && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r5/bench_base.json 2> gpurun_out/r5/bench_base.log
