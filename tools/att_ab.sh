set -o pipefail
O=gpurun_out/att; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_transformer_gpu.py tests/test_latent_full_gpu.py -x -q --timeout 300 --timeout-method thread -k "attention or attn or transformer or psld" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for v in default attold; do
  if [ $v = default ]; then lib=""; else lib=samplers_amd/lib/variants/lib_$v.so; fi
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 200 python -u tools/bench_attention.py > $O/attn_$v.jsonl 2>&1 || exit $?
  echo "== $v"; grep "^{" $O/attn_$v.jsonl | cut -c1-200
done
for v in default attold; do
  if [ $v = default ]; then lib=""; else lib=samplers_amd/lib/variants/lib_$v.so; fi
  env ${lib:+SAMPLERS_HIP_LIB=$lib} timeout -k 10 300 python -u tools/bench_psld.py --steps 3 > $O/psld_$v.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('$O/psld_$v.log').read().strip().splitlines()[-1]); print('$v psld', d['value'], d['ms_per_step'])"
done
