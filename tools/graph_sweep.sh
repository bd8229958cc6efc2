#!/bin/bash
# eager vs hipGraph replay of the DPS step by batch (configs[0]-shaped identity problem):
# the crossover below which DPSSampler replays a captured step by default
set -o pipefail
O=gpurun_out/r5/graph_sweep; mkdir -p $O
for b in ${BATCHES:-1 2 4 8 16 32}; do
  for mode in eager graph; do
    flag=""; [ $mode = graph ] && flag="--graph"
    timeout -k 10 300 python bench.py --config identity --batch $b --steps ${STEPS:-20} --warmup 3 $flag --no-cpu-baseline \
      > $O/b${b}_$mode.json 2> $O/b${b}_$mode.log || exit $?
    python -c "import json;d=json.load(open('$O/b${b}_$mode.json'));print('B=$b $mode', d['ms_per_step'], d['value'])"
  done
done
