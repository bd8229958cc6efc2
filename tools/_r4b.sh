set -o pipefail
O=gpurun_out/r4b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_debug_build_gpu.py -x -v --timeout 500 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/tests.log | head -20; exit $rc; }
timeout -k 10 200 python -u bench.py --config identity --batch 1 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_b1.log 2>&1 || exit 1; tail -1 $O/bench_b1.log | cut -c1-300
timeout -k 10 200 python -u bench.py --steps 5 --no-cpu-baseline > $O/bench_b64.log 2>&1 || exit 1; tail -1 $O/bench_b64.log | cut -c1-300
PARTS="b1" tools/round4_secondary.sh || exit 1
OPS=inpaint timeout -k 10 200 python -u tools/bench_kernels.py > $O/kern_256.log 2>&1 || exit 1
OPS=inpaint IMAGE=512 BATCH=16 timeout -k 10 200 python -u tools/bench_kernels.py > $O/kern_512.log 2>&1 || exit 1
cat $O/kern_256.log $O/kern_512.log
