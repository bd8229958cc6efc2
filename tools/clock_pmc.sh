#!/bin/bash
# Effective shader clock per kernel (GRBM_GUI_ACTIVE / 8 XCDs / kernel time) in the headline step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/clock; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/run -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/run.log 2>&1 || exit $?
ls $O/run
