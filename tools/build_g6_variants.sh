#!/bin/bash
# libsamplers_hip.so variants of the bf16x6 1x1 GEMM (csrc/sp_gemm_x6.hip) for tools/bench_gemm_x6.py:
#   G6_VARIANTS="name:-DFLAG=1,..."   SAMPLERS_HIP_LIB=samplers_amd/lib/variants/lib_g6_<name>.so
set -e
cd "$(dirname "$0")/.."
make -s
mkdir -p build/variants samplers_amd/lib/variants
OTHERS=$(ls build/*.o | grep -v sp_gemm_x6.o)
for v in ${G6_VARIANTS:-"nomfma:-DG6_EXP=1" "nosplit:-DG6_EXP=2" "noload:-DG6_EXP=3"}; do
  name=${v%%:*}; flags=$(echo "${v#*:}" | tr , ' ')
  ( /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -c samplers_amd/csrc/sp_gemm_x6.hip \
      -o build/variants/g6_$name.o &&
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o samplers_amd/lib/variants/lib_g6_$name.so \
      build/variants/g6_$name.o $OTHERS ) &
done
wait
ls samplers_amd/lib/variants
