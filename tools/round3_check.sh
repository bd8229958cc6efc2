#!/bin/bash
# Full GPU suite + headline / blur benches on the current tree (+ optional blur variants).
set -o pipefail
O=gpurun_out/r3; mkdir -p $O
step() { local t=$1 log=$2; shift 2; echo "[r3] $log"; timeout -k 10 $t "$@" > $O/$log 2>&1; local rc=$?; tail -2 $O/$log; [ $rc -eq 0 ] || { echo "[r3] $log failed rc=$rc"; exit $rc; }; }
step 700 gpu_tests.log python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
step 300 bench_inpaint.json python -u bench.py --no-cpu-baseline
step 300 bench_blur.json python -u bench.py --config blur --no-cpu-baseline
if [ -n "$VARIANTS" ]; then bash tools/blur_variants_run.sh; fi
echo "[r3] done"
