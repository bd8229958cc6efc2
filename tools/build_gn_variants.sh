#!/bin/bash
# libsamplers_hip.so variants of the GroupNorm kernels, for
# SAMPLERS_HIP_LIB=samplers_amd/lib/variants/lib_gn_<name>.so python tools/bench_gn.py / bench.py
set -e
cd "$(dirname "$0")/.."
make -s
mkdir -p build/variants samplers_amd/lib/variants
OTHERS=$(ls build/*.o | grep -v sp_groupnorm.o)
# GN_VARIANTS: "name:flags;name:flags;..."
IFS=';' read -ra VARIANTS <<< "${GN_VARIANTS:-team:-DSP_GN_PIPE_FWD=0 -DSP_GN_PIPE_BWD=0}"
for v in "${VARIANTS[@]}"; do
  name=${v%%:*}; flags=${v#*:}
  ( /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -c samplers_amd/csrc/sp_groupnorm.hip \
      -o build/variants/gn_$name.o &&
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o samplers_amd/lib/variants/lib_gn_$name.so \
      build/variants/gn_$name.o $OTHERS ) &
done
wait
ls samplers_amd/lib/variants
