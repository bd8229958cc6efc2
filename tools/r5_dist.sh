set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r5
timeout -k 10 300 python tools/bi_diag.py > gpurun_out/r5/bi_diag.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_distributed_gpu.py tests/test_graph_gpu.py -k "unet or timestep" > gpurun_out/r5/dist_tests.log 2>&1
