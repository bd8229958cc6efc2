#!/bin/bash
# Batch-1 (configs[0] on the GPU) latency work: the split-K tests, the B = 1 eager / hipGraph and
# B = 64 benches, a rocprofv3 kernel trace and a cProfile of the eager B = 1 step's host side.
#   tools/b1_ab.sh  ->  gpurun_out/b1/
set -o pipefail
O=gpurun_out/b1; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gemm_x6_gpu.py tests/test_conv_gpu.py tests/test_transformer_gpu.py tests/test_graph_gpu.py tests/test_debug_build_gpu.py tests/test_latent_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for a in "b1:--config identity --batch 1 --steps 20 --warmup 3" "b1g:--config identity --batch 1 --steps 20 --warmup 3 --graph" "b64:--steps 10"; do
  n=${a%%:*}; args=${a#*:}
  timeout -k 10 200 python -u bench.py $args --no-cpu-baseline > $O/bench_$n.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('$O/bench_$n.log').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
timeout -k 10 200 python -u -m cProfile -o $O/b1.cprof bench.py --config identity --batch 1 --steps 20 --warmup 3 --no-cpu-baseline > $O/cprof_bench.log 2>&1 || exit $?
python -c "import pstats; s=pstats.Stats('$O/b1.cprof'); s.sort_stats('tottime').print_stats(45)" > $O/cprof_tottime.txt
python -c "import pstats; s=pstats.Stats('$O/b1.cprof'); s.sort_stats('cumulative').print_stats(60)" > $O/cprof_cum.txt
R=$(pwd); cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_b1 -o run -- python3 $R/bench.py --config identity --batch 1 --steps 20 --warmup 3 --no-cpu-baseline > $R/$O/prof_b1.log 2>&1
cd $R && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_b64 -o run -- python3 $R/bench.py --steps 5 --no-cpu-baseline > $R/$O/prof_b64.log 2>&1
