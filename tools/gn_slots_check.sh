#!/bin/bash
# GroupNorm self-cleaning team words: the whole GPU test suite, then the DPS step and PSLD with the
# library-owned slot region (default) against lib_gn_memset.so (the caller's workspace zeroed
# every call), and configs[0] (B = 1) both ways.  Output: gpurun_out/gnslots/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/gnslots
mkdir -p $O
cd $R
step() { local t=$1 log=$2; shift 2; echo "[gs] $log"; timeout -k 10 $t "$@" > $O/$log 2>&1; local rc=$?; tail -2 $O/$log; [ $rc -eq 0 ] || { echo "[gs] $log failed rc=$rc"; exit $rc; }; }
step 900 tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/
OLD=$R/samplers_amd/lib/variants/lib_gn_memset.so
step 200 bench_new.log python -u bench.py --no-cpu-baseline
step 200 bench_old.log env SAMPLERS_HIP_LIB=$OLD python -u bench.py --no-cpu-baseline
step 200 b1_new.log python -u bench.py --config identity --batch 1 --steps 20 --warmup 3 --no-cpu-baseline
step 200 b1_old.log env SAMPLERS_HIP_LIB=$OLD python -u bench.py --config identity --batch 1 --steps 20 --warmup 3 --no-cpu-baseline
step 300 psld_new.log python -u tools/bench_psld.py
step 300 psld_old.log env SAMPLERS_HIP_LIB=$OLD python -u tools/bench_psld.py
for f in bench_new bench_old b1_new b1_old psld_new psld_old; do
  echo "== $f $(grep '^{' $O/$f.log | tail -1 | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("groupnorm_recomputed_partials"))')"
done
