#!/bin/bash
# bf16x6 GEMM check after a change: its tests, the headline bench twice, B = 1, and a rocprofv3
# kernel trace of the headline bench (k_gemm_x6 averages) ->  gpurun_out/x6/
set -o pipefail
O=gpurun_out/x6; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_x6_gpu.py tests/test_transformer_gpu.py tests/test_graph_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for a in "b64:--steps 10" "b1:--config identity --batch 1 --steps 20 --warmup 3" "b64b:--steps 10"; do
  n=${a%%:*}; args=${a#*:}
  timeout -k 10 240 python -u bench.py $args --no-cpu-baseline > $O/bench_$n.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('$O/bench_$n.log').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
R=$(pwd); cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_b64 -o run -- python3 $R/bench.py --steps 5 --no-cpu-baseline > $R/$O/prof_b64.log 2>&1
