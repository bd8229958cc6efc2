#!/bin/bash
# configs[0] (B = 1) and the headline step with two GroupNorm builds: the default library
# (self-cleaning words in the library-owned region) and lib_gn_memset.so (the same kernels on the
# caller's workspace, zeroed each call), after the GroupNorm parity tests.  Output: gpurun_out/gnb1/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/gnb1
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_groupnorm_gpu.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in default memset; do
  if [ $v = default ]; then lib=""; else lib=$R/samplers_amd/lib/variants/lib_gn_$v.so; fi
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 200 python -u bench.py --config identity --batch 1 --steps 20 --warmup 3 --no-cpu-baseline > $O/b1_$v.log 2>&1 || exit 1
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 5 > $O/b64_$v.log 2>&1 || exit 1
  echo "$v b1 $(grep '^{' $O/b1_$v.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')  b64 $(grep '^{' $O/b64_$v.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
