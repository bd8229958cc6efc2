#!/bin/bash
# Build libsamplers_hip.so variants of the MFMA convolution tile into build/variants/
#   SAMPLERS_HIP_LIB=build/variants/lib_conv_c4t8.so python tools/bench_conv.py
set -e
cd "$(dirname "$0")/.."
mkdir -p build/variants
SRC="samplers_amd/csrc/sp_dps.hip samplers_amd/csrc/sp_blur.hip samplers_amd/csrc/sp_latent.hip samplers_amd/csrc/sp_groupnorm.hip samplers_amd/csrc/sp_conv.hip samplers_amd/csrc/sp_wino.hip"
VARIANTS=("c4t4:-DSP_CONV_CI=4 -DSP_CONV_TPH=4"
          "c4t8:-DSP_CONV_CI=4 -DSP_CONV_TPH=8"
          "c8t4:-DSP_CONV_CI=8 -DSP_CONV_TPH=4 -DSP_CONV_MINB=1"
          "c8t8:-DSP_CONV_CI=8 -DSP_CONV_TPH=8 -DSP_CONV_MINB=1"
          "c2t8:-DSP_CONV_CI=2 -DSP_CONV_TPH=8")
for v in "${VARIANTS[@]}"; do
  name=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -shared $SRC \
    -o build/variants/lib_conv_$name.so &
done
wait
ls build/variants
