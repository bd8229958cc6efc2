#!/bin/bash
# A/B of the bf16x6 GEMM forms: the default library (register-prefetched X, k_gemm_x6r) against
# lib_g6_old.so (LDS raw-X ring, k_gemm_x6), after the GEMM / transformer parity tests.
# Output: gpurun_out/g6ab/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g6ab
mkdir -p $O
cd $R
step() { local t=$1 log=$2; shift 2; echo "[ab] $log"; timeout -k 10 $t "$@" > $O/$log 2>&1; local rc=$?; tail -2 $O/$log; [ $rc -eq 0 ] || { echo "[ab] $log failed rc=$rc"; exit $rc; }; }
step 300 tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm_x6_gpu.py tests/test_transformer_gpu.py
OLD=$R/samplers_amd/lib/variants/lib_g6_old.so
step 120 gemm_new.log python -u tools/bench_gemm_x6.py
step 120 gemm_old.log env SAMPLERS_HIP_LIB=$OLD python -u tools/bench_gemm_x6.py
step 200 bench_new.log python -u bench.py --no-cpu-baseline
step 200 bench_old.log env SAMPLERS_HIP_LIB=$OLD python -u bench.py --no-cpu-baseline
step 300 psld_new.log python -u tools/bench_psld.py
step 300 psld_old.log env SAMPLERS_HIP_LIB=$OLD python -u tools/bench_psld.py
for f in gemm_new gemm_old; do echo "== $f"; grep "^{" $O/$f.log | python3 -c "import sys,json; [print({k:v for k,v in json.loads(l).items() if 'ms' in k or 'err' in k}) for l in sys.stdin]"; done
for f in bench_new bench_old psld_new psld_old; do echo "== $f"; grep "^{" $O/$f.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; done
