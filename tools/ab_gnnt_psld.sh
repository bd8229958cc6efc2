#!/bin/bash
# bf16 GroupNorm NT policy above 256 MB: loads only / loads + stores / never (the shipped build) — PSLD bf16 and DPS bf16
set -o pipefail
mkdir -p gpurun_out/gnnt3
for v in ntload ntboth base; do
  lib=samplers_amd/lib/libsamplers_hip.so; [ $v = base ] || lib=samplers_amd/lib/variants/lib_$v.so
  SAMPLERS_HIP_LIB=$lib timeout -k 10 400 python -u tools/bench_psld.py --dtype bf16 > gpurun_out/gnnt3/psld_$v.log 2>&1 || exit $?
  SAMPLERS_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --dtype bf16 --no-cpu-baseline > gpurun_out/gnnt3/dps_$v.json 2> gpurun_out/gnnt3/dps_$v.log || exit $?
done
