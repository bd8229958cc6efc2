#!/bin/bash
# GPU check after the attention / GroupNorm hand-over changes: parity tests, the DPS and PSLD
# benches, and the PSLD kernel statistics.  Output: gpurun_out/chk2/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/chk2
mkdir -p $O
cd $R
step() { local t=$1 log=$2; shift 2; echo "[chk] $log"; timeout -k 10 $t "$@" > $O/$log 2>&1; local rc=$?; tail -2 $O/$log; [ $rc -eq 0 ] || { echo "[chk] $log failed rc=$rc"; exit $rc; }; }
step 500 tests.log python -u -m pytest -x -v -s --timeout 120 --timeout-method thread -m gpu \
  tests/test_transformer_gpu.py tests/test_groupnorm_gpu.py tests/test_latent_full_gpu.py tests/test_trajectory_gpu.py
step 200 bench.log python -u bench.py --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
step 300 rocprof_psld.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/psld -o run -- python3 $R/tools/bench_psld.py --steps 3 --warmup 1
echo "[chk] done"
