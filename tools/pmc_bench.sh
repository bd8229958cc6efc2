#!/bin/bash
# HBM traffic of the bench step's kernels: FETCH_SIZE and WRITE_SIZE in separate rocprofv3
# --pmc passes (MI355X_MICROARCH.md: one TCC counter group per pass) over
# `bench.py --config <cfg>`.  Output: gpurun_out/pmc_bench/<cfg>/{fetch,write}/
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for cfg in "$@"; do
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$R/gpurun_out/pmc_bench/$cfg/$(echo $c | cut -d_ -f1 | tr A-Z a-z)
    mkdir -p $d
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $d -o run -- \
      python3 $R/bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > $d.log 2>&1
  done
done
