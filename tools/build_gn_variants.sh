#!/bin/bash
# libsamplers_hip.so variants of the GroupNorm kernels (chunk size per workgroup), for
# SAMPLERS_HIP_LIB=build/variants/lib_gn_<name>.so python bench.py ...
set -e
cd "$(dirname "$0")/.."
make -s
mkdir -p build/variants
OTHERS=$(ls build/*.o | grep -v sp_groupnorm.o)
for v in ${GN_VARIANTS:-"b16k:-DSP_GN_CHUNK_BWD=16384" "f8k:-DSP_GN_CHUNK_FWD=8192"}; do
  name=${v%%:*}; flags=${v#*:}
  ( /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -c samplers_amd/csrc/sp_groupnorm.hip \
      -o build/variants/gn_$name.o &&
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o build/variants/lib_gn_$name.so \
      build/variants/gn_$name.o $OTHERS ) &
done
wait
ls build/variants
