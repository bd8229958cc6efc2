#!/bin/bash
# GPU check of the transformer-glue kernels (LayerNorm / GEGLU / layout GEMMs / strided
# attention), then the PSLD bench and the whole-solve ReSample bench.  Output: gpurun_out/f1/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/f1
mkdir -p $O
cd $R
step() { local t=$1 log=$2; shift 2; echo "[f1] $log: $*"; timeout -k 10 $t "$@" > $O/$log 2>&1; local rc=$?; tail -3 $O/$log; [ $rc -eq 0 ] || { echo "[f1] $log failed rc=$rc"; exit $rc; }; }
step 400 tests.log python -u -m pytest -x -v -s --timeout 120 --timeout-method thread -m gpu \
  tests/test_transformer_gpu.py tests/test_attention_gpu.py tests/test_gemm_x6_gpu.py tests/test_latent_full_gpu.py \
  tests/test_trajectory_gpu.py
[ "${BENCH:-1}" = 1 ] || exit 0
step 200 bench.log python -u bench.py --no-cpu-baseline
step 300 bench_psld.log python -u tools/bench_psld.py
step 420 bench_resample.log python -u tools/bench_resample.py --full-call 20 --max-iters 100 --cpu-baseline
echo "[f1] done"
