#!/bin/bash
# bf16 conv tile: wave-priority variants (SP_CONV_PRIO) against the shipped build, one box
set -o pipefail
mkdir -p gpurun_out/prio
for v in base prio1 prio2; do
  lib=samplers_amd/lib/libsamplers_hip.so; [ $v = base ] || lib=samplers_amd/lib/variants/lib_$v.so
  SAMPLERS_HIP_LIB=$lib timeout -k 10 300 python -u tools/bench_conv_bf16.py --shapes vae --reps 10 > gpurun_out/prio/conv_$v.jsonl 2>&1 || exit $?
done
for v in base prio1 prio2; do
  lib=samplers_amd/lib/libsamplers_hip.so; [ $v = base ] || lib=samplers_amd/lib/variants/lib_$v.so
  SAMPLERS_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --dtype bf16 --no-cpu-baseline > gpurun_out/prio/dps_$v.json 2> gpurun_out/prio/dps_$v.log || exit $?
done
