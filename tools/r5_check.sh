#!/bin/bash
# Round-5 check on the committed tree: the GPU suite, smoke, then the PSLD bench (configs[3]) and
# the ReSample whole-call record (configs[4]) — each step under its own limit, the first failure
# ends the script.  Output: gpurun_out/r5/check/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5/check
mkdir -p $O
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local t=$1 log=$2; shift 2; echo "[check] $log"; timeout -k 10 $t "$@" > $O/$log 2>&1; local rc=$?; tail -1 $O/$log | cut -c1-200; [ $rc -eq 0 ] || { echo "[check] $log failed rc=$rc"; tail -5 $O/$log; exit $rc; }; }
[ -z "$SKIP_TESTS" ] && step 1000 gpu_tests.log python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread
[ -z "$SKIP_TESTS" ] && step 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
[ -n "$PSLD" ] && step 400 bench_psld.log python -u tools/bench_psld.py --cpu-baseline
[ -n "$RESAMPLE" ] && step 1100 bench_resample_whole.log python -u tools/bench_resample.py --batch 32 --steps 3 --warmup 2 --pixel-iters 2000 --latent-iters 200 --cpu-baseline --heartbeat $O/rs_heartbeat.log
echo "[check] done"
