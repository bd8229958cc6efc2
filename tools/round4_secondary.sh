#!/bin/bash
# Round-4 secondary measurements, one GPU step each under its own limit (the first failure ends
# the script).  PART=debug: the bounds-checked debug build test; PART=b1: a rocprofv3 kernel
# profile of the B = 1 identity step (configs[0] on the GPU); PART=resample: one whole ReSample
# solve at the reference's defaults (100 steps, max_optimization_iters 2000, time travel every
# 10) at batch 2; PART=psld: PSLD without CFG with its CPU baseline.
# Output: gpurun_out/r4/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4
mkdir -p $O
cd $R
step() { local t=$1 log=$2; shift 2; echo "[r4] $log"; timeout -k 10 $t "$@" > $O/$log 2>&1; local rc=$?; tail -1 $O/$log | cut -c1-200; [ $rc -eq 0 ] || { echo "[r4] $log failed rc=$rc"; tail -20 $O/$log; exit $rc; }; }
for part in ${PARTS:-debug b1 resample psld}; do
  case $part in
    debug) step 600 debug_tests.log python -u -m pytest tests/test_debug_build_gpu.py -x -v --timeout 600 --timeout-method thread ;;
    b1) (cd /tmp && export TMPDIR=/tmp && step 300 rocprof_b1.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b1 -o run -- python3 $R/bench.py --config identity --batch 1 --steps 20 --warmup 3 --no-cpu-baseline) || exit 1 ;;
    resample) step 1100 bench_resample_full.log python -u tools/bench_resample.py --batch 2 --full-batch 1 --steps 2 --warmup 1 --full-call 100 --max-iters 2000 --time-travel-interval 10 ;;
    psld) step 400 bench_psld_cpu.log python -u tools/bench_psld.py --cpu-baseline ;;
  esac
done
echo "[r4] done"
