#!/bin/bash
# Eager vs hipGraph replay of the DPS step (bench.py --graph) on one box: the inter-kernel gaps
# (~4.8 us median per boundary in rocprofv3 traces, ~520 launches per step) are what replay saves.
#   tools/graph_ab.sh  ->  gpurun_out/graph/
set -o pipefail
O=gpurun_out/graph; mkdir -p $O
for a in "b64:--steps 10" "b64g:--steps 10 --graph" "b1:--config identity --batch 1 --steps 20 --warmup 3" "b1g:--config identity --batch 1 --steps 20 --warmup 3 --graph" "b512g:--image 512 --batch 16 --steps 5 --graph"; do
  n=${a%%:*}; args=${a#*:}
  timeout -k 10 240 python -u bench.py $args --no-cpu-baseline > $O/bench_$n.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('$O/bench_$n.log').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
