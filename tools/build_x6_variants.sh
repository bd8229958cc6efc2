#!/bin/bash
# libsamplers_hip.so variants of the bf16x6 Winograd tile (csrc/sp_wino_x6.hip rebuilt with each
# knob, linked with the other objects of `make`) for tools/bench_x6.py:
#   X6_VARIANTS="name:-DFLAG=1,-DOTHER=0 ..."   SAMPLERS_HIP_LIB=samplers_amd/lib/variants/lib_x6_<name>.so
set -e
cd "$(dirname "$0")/.."
make -s
mkdir -p build/variants samplers_amd/lib/variants
OTHERS=$(ls build/*.o | grep -v sp_wino_x6.o)
for v in ${X6_VARIANTS:-"noload:-DX6_EXP=1" "nomfma:-DX6_EXP=2" "nowait:-DX6_EXP=3"}; do
  name=${v%%:*}; flags=$(echo "${v#*:}" | tr , ' ')
  ( /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -c samplers_amd/csrc/sp_wino_x6.hip \
      -o build/variants/x6_$name.o &&
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o samplers_amd/lib/variants/lib_x6_$name.so \
      build/variants/x6_$name.o $OTHERS ) &
done
wait
ls samplers_amd/lib/variants
