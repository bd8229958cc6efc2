set -e
export CUSTOM="64,128,128,256,256;64,256,256,128,128"
timeout -k 10 120 python -u tools/bench_conv_x6.py > gpurun_out/c6v_base.jsonl 2>&1
for v in nomfma nosplit noload bar9 late1 late2 late4; do
  SAMPLERS_HIP_LIB=samplers_amd/lib/variants/lib_c6_$v.so timeout -k 10 120 python -u tools/bench_conv_x6.py > gpurun_out/c6v_$v.jsonl 2>&1
done
