#!/bin/bash
# Headline bench with GroupNorm variants: two-pass, single-pass (chunk 16k, 8k, 4k).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/gnv
mkdir -p $O
cd $R
run() {
  timeout -k 10 240 env "$@" python bench.py --no-cpu-baseline --steps 5 > $O/$name.json 2> $O/$name.err
  python -c "import json; d=json.load(open('$O/$name.json')); print('$name', d['value'], d['ms_per_step'])"
}
name=twopass; run SAMPLERS_AMD_GN_SINGLE_PASS=0
name=c16k; run SAMPLERS_AMD_GN_SINGLE_PASS=1
name=c8k; run SAMPLERS_HIP_LIB=build/variants/lib_gn_c8k.so
name=c4k; run SAMPLERS_HIP_LIB=build/variants/lib_gn_c4k.so
name=c4k_twopass; run SAMPLERS_HIP_LIB=build/variants/lib_gn_c4k.so SAMPLERS_AMD_GN_SINGLE_PASS=0
