set -o pipefail
O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_latent_full_gpu.py tests/test_attention_gpu.py tests/test_trajectory_gpu.py -x -q --timeout 300 --timeout-method thread -k "not long" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head; exit $rc; }
timeout -k 10 200 python -u bench.py --config identity --batch 1 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_b1.log 2>&1 || exit 1; tail -1 $O/bench_b1.log | cut -c1-200
timeout -k 10 200 python -u bench.py --config identity --batch 1 --steps 20 --warmup 3 --no-cpu-baseline --graph > $O/bench_b1_graph.log 2>&1 || exit 1; tail -1 $O/bench_b1_graph.log | cut -c1-200
timeout -k 10 200 python -u bench.py --steps 5 --no-cpu-baseline > $O/bench_b64.log 2>&1 || exit 1; tail -1 $O/bench_b64.log | cut -c1-200
timeout -k 10 300 python -u bench.py --image 512 --batch 16 --steps 5 --no-cpu-baseline > $O/bench_512.log 2>&1 || exit 1; tail -1 $O/bench_512.log | cut -c1-200
