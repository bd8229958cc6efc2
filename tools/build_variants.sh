#!/bin/bash
# Build libsamplers_hip.so variants (tuning knobs) into build/variants/ for tools/bench_kernels.py
set -e
cd "$(dirname "$0")/.."
mkdir -p build/variants
for v in "k4:-DSP_KITER=4" "k6:-DSP_KITER=6" "k8:-DSP_KITER=8" "k4nt:-DSP_KITER=4 -DSP_NT_STORE=1" "k8nt:-DSP_KITER=8 -DSP_NT_STORE=1" "k2:-DSP_KITER=2"; do
  name=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -shared \
    samplers_amd/csrc/sp_dps.hip samplers_amd/csrc/sp_blur.hip samplers_amd/csrc/sp_latent.hip -o build/variants/lib_$name.so &
done
wait
ls build/variants
