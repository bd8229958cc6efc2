#!/bin/bash
# bf16 GroupNorm streams: non-temporal loads + stores above a size threshold (SP_GNB_NT_MB: shipped 256,
# variants never / 64) — tools/bench_gn_bf16.py and the DPS bf16 step, one box
set -o pipefail
mkdir -p gpurun_out/gnnt2
for v in base ntnever nt64; do
  lib=samplers_amd/lib/libsamplers_hip.so; [ $v = base ] || lib=samplers_amd/lib/variants/lib_$v.so
  SAMPLERS_HIP_LIB=$lib timeout -k 10 300 python -u tools/bench_gn_bf16.py > gpurun_out/gnnt2/gn_$v.log 2>&1 || exit $?
  SAMPLERS_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --dtype bf16 --no-cpu-baseline > gpurun_out/gnnt2/dps_$v.json 2> gpurun_out/gnnt2/dps_$v.log || exit $?
done
