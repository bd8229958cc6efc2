#!/bin/bash
# Kernel-time breakdown of the PSLD / ReSample benches (BASELINE configs[3] / [4]).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/latent; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/psld -o run -- python3 $R/tools/bench_psld.py --steps 2 --warmup 1 > $O/psld.log 2>&1 || exit $?
tail -1 $O/psld.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/resample -o run -- python3 $R/tools/bench_resample.py --steps 2 --warmup 1 > $O/resample.log 2>&1 || exit $?
tail -1 $O/resample.log | cut -c1-200
ls $O/psld $O/resample
