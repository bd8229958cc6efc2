#!/bin/bash
# One round's GPU measurements, in two gpurun calls (each under gpurun's 20-minute limit):
#   bash tools/round3_measure.sh benches   headline bench (with the CPU baseline), blur and 512²
#                                          DPS records, PSLD (CFG on) / ReSample (whole solve) on
#                                          the SD 1.5 priors with their CPU baselines
#   bash tools/round3_measure.sh profiles  the bench and PSLD under rocprofv3 --kernel-trace
#                                          --stats, and the FETCH_SIZE / WRITE_SIZE passes
# Output: gpurun_out/measure3/.  Every GPU step has its own time limit; the first failure ends
# the script.
set -o pipefail
PART=${1:-benches}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/measure3
mkdir -p $O
cd $R
step() { local t=$1 log=$2; shift 2; echo "[measure] $log: $*"; timeout -k 10 $t "$@" > $O/$log 2>&1; local rc=$?; tail -2 $O/$log; [ $rc -eq 0 ] || { echo "[measure] $log failed rc=$rc"; exit $rc; }; }
(nproc; echo OMP=$OMP_NUM_THREADS; cat /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpuset.cpus.effective 2>&1; lscpu | head -20) > $O/host.txt 2>&1
if [ "$PART" = benches ]; then
  step 300 bench_inpaint.log python -u bench.py
  step 200 bench_blur.log python -u bench.py --config blur --no-cpu-baseline
  step 200 bench_inpaint_512_b16.log python -u bench.py --image 512 --batch 16 --no-cpu-baseline
  step 300 bench_psld_cfg_b32_512.log python -u tools/bench_psld.py --cfg --cpu-baseline
  step 420 bench_resample_b32_512.log python -u tools/bench_resample.py --full-call 20 --max-iters 100 --cpu-baseline
else
  cd /tmp && export TMPDIR=/tmp
  step 300 rocprof_stats.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 5 --no-cpu-baseline
  step 300 rocprof_psld.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_psld -o run -- python3 $R/tools/bench_psld.py --steps 3 --warmup 1
  for cfg in inpaint blur; do
    for c in FETCH_SIZE WRITE_SIZE; do
      step 240 pmc_${cfg}_$c.log rocprofv3 --pmc $c --output-format csv -d $O/pmc/$cfg/$c -o run -- python3 $R/bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline
    done
  done
fi
echo "[measure] $PART done"
