#!/bin/bash
# libsamplers_hip.so variants of the blur DPS pass for tools/bench_kernels.py (OPS=blur):
# sp_blur.hip rebuilt with each knob, linked with the other objects of `make`.
#   BLUR_VARIANTS="name:-DFLAG=1,-DOTHER=0 ..."   (flags of one variant separated by commas)
set -e
cd "$(dirname "$0")/.."
make -s
mkdir -p build/variants samplers_amd/lib/variants
OTHERS=$(ls build/*.o | grep -v sp_blur.o)
for v in ${BLUR_VARIANTS:-"tile:-DSP_BLUR_STREAM=0" "seg32:-DSP_BLUR_SEG=32" "seg64:-DSP_BLUR_SEG=64"}; do
  name=${v%%:*}; flags=$(echo "${v#*:}" | tr , ' ')
  ( /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -c samplers_amd/csrc/sp_blur.hip \
      -o build/variants/blur_$name.o &&
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o samplers_amd/lib/variants/lib_blur_$name.so \
      build/variants/blur_$name.o $OTHERS ) &
done
wait
ls samplers_amd/lib/variants
