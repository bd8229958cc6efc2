#!/bin/bash
# stride-2 conv variants (tools/build_variant.sh NAME ...) against the default library:
#   VARIANTS="s2old" tools/s2_ab.sh  ->  gpurun_out/s2/
set -o pipefail
O=gpurun_out/s2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 200 --timeout-method thread -k "s2 or stride2 or downsample" > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for v in default ${VARIANTS}; do
  if [ $v = default ]; then lib=""; else lib=samplers_amd/lib/variants/lib_$v.so; fi
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 200 python -u tools/bench_s2.py > $O/s2_$v.jsonl 2>&1 || exit $?
  echo "== $v"; grep "^{" $O/s2_$v.jsonl | grep -v upsample | cut -c1-150
done
