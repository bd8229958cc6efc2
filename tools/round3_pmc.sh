#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one counter per run, each under its own time limit) of the
# headline bench, inpaint and blur, for profiles/pmc_traffic.json (tools/pmc_summary.py).
# Output: gpurun_out/pmc3/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc3
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for cfg in inpaint blur; do
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "[pmc] $cfg $c"
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/$cfg/$c -o run -- python3 $R/bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > $O/${cfg}_$c.log 2>&1 || { echo "[pmc] $cfg $c failed"; tail -5 $O/${cfg}_$c.log; exit 1; }
  done
done
echo "[pmc] done"
