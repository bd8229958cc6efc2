#!/bin/bash
# Held clock and MFMA busy of the Winograd tile (tools/wino_clock.py: ~2 s of back-to-back
# forwards on one shape) in the shipped build and its diagnostic builds (SP_WINO_EXP 1: no k-loop
# loads, 2: no output stores, 3: no input transform; tools/build_variant.sh wx1 "-DSP_WINO_EXP=1" ...):
# which part of the tile's work lowers the clock the chip holds (fp32 MFMAs alone hold 2.38 GHz,
# profiles/round5/mfma_power.jsonl).   tools/wino_clock.sh  ->  gpurun_out/wino_clock/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/wino_clock; mkdir -p $O
SHAPE=${SHAPE:-"64 128 128 256 256"}
for v in ${VARIANTS:-default wx1 wx2 wx3}; do
  if [ $v = default ]; then lib=""; else lib=$R/samplers_amd/lib/variants/lib_$v.so; fi
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 120 python3 -u $R/tools/wino_clock.py $SHAPE 800 > $O/time_$v.json 2>&1 || exit $?
  env ${lib:+SAMPLERS_HIP_LIB=$lib} FILTER=k_wino3x3 NAME=wino_$v timeout -k 10 400 bash $R/tools/sq_pmc.sh tools/wino_clock.py $SHAPE 400 > $O/sq_$v.txt 2>&1 || exit $?
  echo "== $v"; cat $O/time_$v.json; grep -h "k_wino" $O/sq_$v.txt | cut -c1-200
done
