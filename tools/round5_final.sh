#!/bin/bash
# Final round-5 measurements on the committed tree (one step per GPU run, each under its own
# limit; the first failure ends the script).  Output: gpurun_out/final5/.
#   PART=benches   the DPS bench records (headline with its CPU baseline, blur, 512² at B = 16 and
#                  24, B = 1 eager and hipGraph, a whole 1000-step B = 1 call at its defaults) and
#                  2- / 8-rank self-launch rehearsals over gloo
#   PART=latent    PSLD with / without CFG and their CPU baselines, ReSample pieces + the
#                  whole-call projection at the reference's defaults
#   PART=pmc       FETCH_SIZE / WRITE_SIZE passes (one counter per run) of the inpaint, blur and
#                  512² benches for profiles/pmc_traffic.json (tools/pmc_summary.py)
#   PART=profiles  rocprofv3 kernel statistics of the DPS (B = 64 and B = 1) and PSLD benches
set -o pipefail
PART=${1:-benches}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/final5
mkdir -p $O
cd $R
step() { local t=$1 log=$2; shift 2; echo "[final] $log"; timeout -k 10 $t "$@" > $O/$log 2>&1; local rc=$?; tail -1 $O/$log | cut -c1-160; [ $rc -eq 0 ] || { echo "[final] $log failed rc=$rc"; tail -5 $O/$log; exit $rc; }; }
if [ "$PART" = benches ]; then
  step 300 bench_inpaint.log python -u bench.py
  step 200 bench_blur.log python -u bench.py --config blur --no-cpu-baseline
  step 200 bench_inpaint_512_b16.log python -u bench.py --image 512 --batch 16 --no-cpu-baseline
  step 300 bench_inpaint_512_b24.log python -u bench.py --image 512 --batch 24 --steps 3 --no-cpu-baseline
  step 200 bench_identity_b1.log python -u bench.py --config identity --batch 1 --steps 20 --warmup 3 --no-cpu-baseline
  step 200 bench_identity_b1_graph.log python -u bench.py --config identity --batch 1 --steps 20 --warmup 3 --no-cpu-baseline --graph
  step 300 bench_call_b1.log python -u tools/bench_call.py --batch 1 --steps 1000
  step 300 bench_gloo2.log env SAMPLERS_AMD_DIST_BACKEND=gloo python -u bench.py --gpus 2 --batch 16 --steps 3 --warmup 1 --no-cpu-baseline
  step 300 bench_gloo8_blur.log env SAMPLERS_AMD_DIST_BACKEND=gloo python -u bench.py --config blur --gpus 8 --batch 2 --steps 3 --warmup 1 --no-cpu-baseline
elif [ "$PART" = latent ]; then
  step 400 bench_psld.log python -u tools/bench_psld.py --cpu-baseline
  step 400 bench_psld_cfg.log python -u tools/bench_psld.py --cfg --cpu-baseline
  step 1100 bench_resample.log python -u tools/bench_resample.py --cpu-baseline --pixel-iters 2000 --latent-iters 200 --heartbeat $O/rs_heartbeat.log
elif [ "$PART" = pmc ]; then
  cd /tmp && export TMPDIR=/tmp
  for cfg in "inpaint:--config inpaint" "blur:--config blur" "inpaint512:--image 512 --batch 16"; do
    name=${cfg%%:*}; args=${cfg#*:}
    for c in FETCH_SIZE WRITE_SIZE; do
      echo "[pmc] $name $c"
      timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/pmc/$name/$c -o run -- python3 $R/bench.py $args --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_${name}_$c.log 2>&1 || { echo "[pmc] $name $c failed"; tail -5 $O/pmc_${name}_$c.log; exit 1; }
    done
  done
else
  cd /tmp && export TMPDIR=/tmp
  step 300 rocprof_bench.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 $R/bench.py --steps 5 --no-cpu-baseline
  step 300 rocprof_b1.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b1 -o run -- python3 $R/bench.py --config identity --batch 1 --steps 20 --warmup 3 --no-cpu-baseline
  step 300 rocprof_psld.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_psld -o run -- python3 $R/tools/bench_psld.py --steps 3 --warmup 1
  cd $R
  step 400 sq_x6.log env FILTER=k_gemm_x6 NAME=x6 bash tools/sq_pmc.sh tools/bench_gemm_x6.py
  step 400 sq_bench.log env FILTER=k_wino3x3 NAME=bench bash tools/sq_pmc.sh bench.py --steps 2 --warmup 1 --no-cpu-baseline
fi
echo "[final] $PART done"
