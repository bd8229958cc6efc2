#!/bin/bash
# rocprofv3 kernel statistics of the DPS bench and the PSLD bench (the sp:: share of PSLD
# kernel time), after the x6 GEMM diagnostics.  Output: gpurun_out/prof3/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof3
mkdir -p $O
cd $R
[ "${DIAG:-1}" = 1 ] && { bash tools/g6_diag.sh || exit 1; }
cd /tmp && export TMPDIR=/tmp
step() { local t=$1 log=$2; shift 2; echo "[prof] $log"; timeout -k 10 $t "$@" > $O/$log 2>&1; local rc=$?; tail -2 $O/$log; [ $rc -eq 0 ] || { echo "[prof] $log failed rc=$rc"; exit $rc; }; }
step 300 rocprof_psld.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/psld -o run -- python3 $R/tools/bench_psld.py --steps 3 --warmup 1
step 300 rocprof_bench.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench -o run -- python3 $R/bench.py --steps 5 --no-cpu-baseline
echo "[prof] done"
