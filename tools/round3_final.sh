#!/bin/bash
# Final round-3 measurements on the committed tree (one step per GPU run, each under its own
# limit; the first failure ends the script).  PART=benches: every bench record and a 2-rank
# self-launch rehearsal over gloo (PART=rest: all but the headline inpaint record); PART=profiles: rocprofv3 kernel statistics of the DPS and PSLD
# benches.  Output: gpurun_out/final3/.
set -o pipefail
PART=${1:-benches}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/final3
mkdir -p $O
cd $R
step() { local t=$1 log=$2; shift 2; echo "[final] $log"; timeout -k 10 $t "$@" > $O/$log 2>&1; local rc=$?; tail -1 $O/$log | cut -c1-160; [ $rc -eq 0 ] || { echo "[final] $log failed rc=$rc"; exit $rc; }; }
if [ "$PART" = benches ] || [ "$PART" = rest ]; then
  [ "$PART" = benches ] && step 300 bench_inpaint.log python -u bench.py
  step 200 bench_blur.log python -u bench.py --config blur --no-cpu-baseline
  step 200 bench_inpaint_512_b16.log python -u bench.py --image 512 --batch 16 --no-cpu-baseline
  step 200 bench_psld.log python -u tools/bench_psld.py
  step 300 bench_psld_cfg.log python -u tools/bench_psld.py --cfg --cpu-baseline
  step 420 bench_resample.log python -u tools/bench_resample.py --full-call 20 --max-iters 100 --cpu-baseline
  step 300 bench_gloo2.log env SAMPLERS_AMD_DIST_BACKEND=gloo python -u bench.py --gpus 2 --batch 16 --steps 3 --warmup 1 --no-cpu-baseline
else
  cd /tmp && export TMPDIR=/tmp
  step 300 rocprof_bench.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 $R/bench.py --steps 5 --no-cpu-baseline
  step 300 rocprof_psld.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_psld -o run -- python3 $R/tools/bench_psld.py --steps 3 --warmup 1
fi
echo "[final] $PART done"
