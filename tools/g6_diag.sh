#!/bin/bash
# Time the bf16x6 GEMM (tools/bench_gemm_x6.py) on the default library and the diagnostic
# variants built by tools/build_g6_variants.sh.  Output: gpurun_out/g6diag/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g6diag
mkdir -p $O
cd $R
for v in default ${G6_LIST:-nomfma nosplit noload nostore}; do
  if [ $v = default ]; then lib=samplers_amd/lib/libsamplers_hip.so; else lib=samplers_amd/lib/variants/lib_g6_$v.so; fi
  SAMPLERS_HIP_LIB=$R/$lib timeout -k 10 120 python -u tools/bench_gemm_x6.py > $O/$v.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.log; exit 1; }
  echo "== $v"; grep "^{" $O/$v.log | python3 -c "import sys,json; [print({k:v for k,v in json.loads(l).items() if 'ms' in k}) for l in sys.stdin]"
done
