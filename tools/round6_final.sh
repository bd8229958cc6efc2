#!/bin/bash
# Final round-6 measurements on the committed tree (one step per GPU run, each under its own
# limit; the first failure ends the script).  Output: gpurun_out/final6/.  Every single-GPU
# record carries its CPU baseline (the oracle on the box's host cores, same workload).
#   PART=benches   DPS bench records: headline inpaint, blur, identity B = 1 (eager and hipGraph),
#                  512² at B = 16
#   PART=latent    PSLD fp32 / bf16 (with and without CFG) with their CPU baselines
#   PART=bf16      PSLD bf16 (with / without CFG) and its rocprofv3 statistics again (the bf16 tiles' late changes)
#   PART=bf16a     DPS bf16 record + rocprofv3 statistics of DPS bf16 and PSLD bf16; PART=bf16b: PSLD bf16 records
#   PART=resample  ReSample pieces + the whole-call projection with its CPU baseline
#   PART=dist      2- / 8-rank self-launch rehearsals over gloo and a whole 1000-step B = 1 call
#   PART=profiles  rocprofv3 kernel statistics of the DPS (B = 64, B = 1) and PSLD fp32 / bf16 benches
set -o pipefail
PART=${1:-benches}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/final6
mkdir -p $O
cd $R
step() { local t=$1 log=$2; shift 2; echo "[final] $log"; timeout -k 10 $t "$@" > $O/$log 2>&1; local rc=$?; tail -1 $O/$log | cut -c1-160; [ $rc -eq 0 ] || { echo "[final] $log failed rc=$rc"; tail -5 $O/$log; exit $rc; }; }
if [ "$PART" = benches ]; then
  step 300 bench_inpaint.log python -u bench.py
  step 300 bench_blur.log python -u bench.py --config blur
  step 300 bench_identity_b1.log python -u bench.py --config identity --batch 1 --steps 20 --warmup 3
  step 300 bench_identity_b1_graph.log python -u bench.py --config identity --batch 1 --steps 20 --warmup 3 --graph
  step 400 bench_inpaint_512_b16.log python -u bench.py --image 512 --batch 16
elif [ "$PART" = latent ]; then
  step 400 bench_psld.log python -u tools/bench_psld.py --cpu-baseline
  step 400 bench_psld_bf16.log python -u tools/bench_psld.py --dtype bf16 --cpu-baseline
  step 400 bench_psld_cfg.log python -u tools/bench_psld.py --cfg --cpu-baseline
  step 400 bench_psld_bf16_cfg.log python -u tools/bench_psld.py --dtype bf16 --cfg --cpu-baseline
elif [ "$PART" = bf16 ]; then
  step 400 bench_psld_bf16.log python -u tools/bench_psld.py --dtype bf16 --cpu-baseline
  step 400 bench_psld_bf16_cfg.log python -u tools/bench_psld.py --dtype bf16 --cfg --cpu-baseline
  cd /tmp && export TMPDIR=/tmp
  step 300 rocprof_psld_bf16.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_psld_bf16 -o run -- python3 $R/tools/bench_psld.py --dtype bf16 --steps 3 --warmup 1
  step 300 rocprof_dps_bf16.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dps_bf16 -o run -- python3 $R/bench.py --dtype bf16 --no-cpu-baseline
  cd $R
  step 400 bench_dps_bf16.log python -u bench.py --dtype bf16
  step 400 bench_psld_bf16_gloo2.log env SAMPLERS_AMD_DIST_BACKEND=gloo python -u tools/bench_psld.py --gpus 2 --dtype bf16 --batch 8 --steps 2 --warmup 1
elif [ "$PART" = bf16a ]; then
  step 400 bench_dps_bf16.log python -u bench.py --dtype bf16
  cd /tmp && export TMPDIR=/tmp
  step 300 rocprof_dps_bf16.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dps_bf16 -o run -- python3 $R/bench.py --dtype bf16 --no-cpu-baseline
  step 300 rocprof_psld_bf16.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_psld_bf16 -o run -- python3 $R/tools/bench_psld.py --dtype bf16 --steps 3 --warmup 1
elif [ "$PART" = bf16b ]; then
  step 400 bench_psld_bf16.log python -u tools/bench_psld.py --dtype bf16 --cpu-baseline
  step 400 bench_psld_bf16_cfg.log python -u tools/bench_psld.py --dtype bf16 --cfg --cpu-baseline
elif [ "$PART" = resample ]; then
  step 1100 bench_resample.log python -u tools/bench_resample.py --cpu-baseline --pixel-iters 2000 --latent-iters 200 --heartbeat $O/rs_heartbeat.log
elif [ "$PART" = dist ]; then
  step 300 bench_call_b1.log python -u tools/bench_call.py --batch 1 --steps 1000
  step 300 bench_gloo2.log env SAMPLERS_AMD_DIST_BACKEND=gloo python -u bench.py --gpus 2 --batch 16 --steps 3 --warmup 1
  step 300 bench_gloo8_blur.log env SAMPLERS_AMD_DIST_BACKEND=gloo python -u bench.py --config blur --gpus 8 --batch 2 --steps 3 --warmup 1
else
  cd /tmp && export TMPDIR=/tmp
  step 300 rocprof_bench.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 $R/bench.py --steps 5 --no-cpu-baseline
  step 300 rocprof_b1.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b1 -o run -- python3 $R/bench.py --config identity --batch 1 --steps 20 --warmup 3 --no-cpu-baseline
  step 300 rocprof_psld.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_psld -o run -- python3 $R/tools/bench_psld.py --steps 3 --warmup 1
  step 300 rocprof_psld_bf16.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_psld_bf16 -o run -- python3 $R/tools/bench_psld.py --dtype bf16 --steps 3 --warmup 1
fi
echo "[final] $PART done"
