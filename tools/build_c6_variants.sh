#!/bin/bash
# libsamplers_hip.so variants of the direct bf16x6 3x3 conv (csrc/sp_gemm_x6.hip, k_conv3x3_x6) for
# tools/bench_conv_x6.py:  C6_VARIANTS="name:-DFLAG=1,..."
#   SAMPLERS_HIP_LIB=samplers_amd/lib/variants/lib_c6_<name>.so python tools/bench_conv_x6.py
set -e
cd "$(dirname "$0")/.."
make -s
mkdir -p build/variants samplers_amd/lib/variants
OTHERS=$(ls build/*.o | grep -v sp_gemm_x6.o)
for v in ${C6_VARIANTS:-"nomfma:-DC6_EXP=1" "nosplit:-DC6_EXP=2" "noload:-DC6_EXP=3" "noread:-DC6_EXP=4" "bar9:-DC6_EXP=5"}; do
  name=${v%%:*}; flags=$(echo "${v#*:}" | tr , ' ')
  ( /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -c samplers_amd/csrc/sp_gemm_x6.hip \
      -o build/variants/c6_$name.o &&
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o samplers_amd/lib/variants/lib_c6_$name.so \
      build/variants/c6_$name.o $OTHERS ) &
done
wait
ls samplers_amd/lib/variants
