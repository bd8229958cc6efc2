#!/bin/bash
# Round 5 A/B of the bf16x6 GEMM's wave layout (verdict item 3): the shipped 8 waves x (64 x 64)
# against G6_W4 (4 waves, one per SIMD, each 128 channels x 64 pixels: no split of an X value by
# two waves, W fragments read at the start of their own step), plus the MFMA-only diagnostic
# builds of both (G6_EXP=6: no loads, no split, no stores) for the structure's floor, and the
# headline step with each wave layout.
#   tools/build_variant.sh w4 "-DG6_W4=1"; tools/build_variant.sh e6 "-DG6_EXP=6"
#   tools/build_variant.sh w4e6 "-DG6_W4=1 -DG6_EXP=6"; tools/x6_w4_ab.sh  ->  gpurun_out/x6w4/
set -o pipefail
O=gpurun_out/x6w4; mkdir -p $O
V=samplers_amd/lib/variants
SAMPLERS_HIP_LIB=$V/lib_w4.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_x6_gpu.py > $O/w4_tests.log 2>&1 || exit $?
for v in default w4 e6 w4e6; do
  if [ $v = default ]; then lib=""; else lib=$V/lib_$v.so; fi
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 200 python -u tools/bench_gemm_x6.py > $O/gemm_$v.jsonl 2>&1 || exit $?
  echo "== $v"; grep -h "x6" $O/gemm_$v.jsonl | cut -c1-200 | head -4
done
for v in default w4 default w4; do
  if [ $v = default ]; then lib=""; else lib=$V/lib_$v.so; fi
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.log || exit $?
  echo "== bench $v"; cut -c1-160 $O/bench_$v.json
done
