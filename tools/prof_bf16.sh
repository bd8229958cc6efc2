#!/bin/bash
# rocprofv3 kernel statistics of the bf16 PSLD (configs[3]) and DPS (B = 64, 256^2) benches:
# gpurun_out/prof7/{psld,dps}/run_kernel_stats.csv (one kernel-trace run each, no counters)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof7
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/psld -o run -- python3 $R/tools/bench_psld.py --dtype bf16 > $O/psld.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dps -o run -- python3 $R/bench.py --dtype bf16 --no-cpu-baseline > $O/dps.log 2>&1
