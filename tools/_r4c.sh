set -o pipefail
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_dps_gpu.py tests/test_full_size_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
OPS=inpaint IMAGE=512 BATCH=16 timeout -k 10 200 python -u tools/bench_kernels.py > $O/kern_512.log 2>&1 || exit 1
OPS=inpaint,blur timeout -k 10 200 python -u tools/bench_kernels.py > $O/kern_256.log 2>&1 || exit 1
cat $O/kern_512.log $O/kern_256.log | grep -v amdgpu.ids
timeout -k 10 200 python -u tools/bench_score_gemm.py > $O/score_gemm.log 2>&1 || exit 1
grep -v amdgpu.ids $O/score_gemm.log
