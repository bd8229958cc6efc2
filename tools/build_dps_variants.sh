#!/bin/bash
# libsamplers_hip.so variants of the DPS passes (sp_dps.hip rebuilt per knob, linked with the
# other objects of `make`) for tools/bench_kernels.py:  DPS_VARIANTS="name:-DFLAG=1,-DX=2 ..."
set -e
cd "$(dirname "$0")/.."
make -s
mkdir -p build/variants samplers_amd/lib/variants
OTHERS=$(ls build/*.o | grep -v sp_dps.o)
for v in $DPS_VARIANTS; do
  name=${v%%:*}; flags=$(echo "${v#*:}" | tr , ' ')
  ( /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -c samplers_amd/csrc/sp_dps.hip \
      -o build/variants/dps_$name.o &&
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o samplers_amd/lib/variants/lib_dps_$name.so \
      build/variants/dps_$name.o $OTHERS ) &
done
wait
ls samplers_amd/lib/variants
