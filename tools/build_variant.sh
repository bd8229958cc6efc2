#!/bin/bash
# Build a variant of libsamplers_hip.so with extra compile-time knobs (A/B measurements):
#   tools/build_variant.sh NAME "-DKNOB=VALUE ..."  ->  samplers_amd/lib/variants/lib_NAME.so
# then e.g.  SAMPLERS_HIP_LIB=samplers_amd/lib/variants/lib_NAME.so python bench.py
# (tools/wino_ab.sh runs the headline bench over a list of them: VARIANTS="a b" tools/wino_ab.sh)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
flags="$*"
out=samplers_amd/lib/variants
mkdir -p $out build/variants/$name
objs=()
for src in $(make -s -p -n 2>/dev/null | sed -n 's/^SRC := //p'); do
  o=build/variants/$name/$(basename ${src%.hip}).o
  # the Makefile's per-file flags
  extra=""; case "$(basename $src)" in
    sp_wino.hip) extra="-fno-slp-vectorize" ;;
    sp_attention.hip|sp_attention6.hip|sp_bf16.hip) extra="-mllvm -amdgpu-mfma-vgpr-form=1" ;;
  esac
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $extra $flags -c $src -o $o &
  objs+=($o)
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $out/lib_$name.so "${objs[@]}"
echo "$out/lib_$name.so"
