#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the blur residual pass per library variant (bench_kernels OPS=blur).
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/pmcblur; mkdir -p $O
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for v in $VARIANTS; do
  for c in FETCH_SIZE WRITE_SIZE; do
    SAMPLERS_HIP_LIB=$R/samplers_amd/lib/variants/lib_blur_$v.so OPS=blur timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/$v/$c -o run -- python3 $R/tools/bench_kernels.py $v > $O/$v.$c.log 2>&1 || { echo "$v $c failed"; tail -5 $O/$v.$c.log; exit 1; }
  done
done
echo done
