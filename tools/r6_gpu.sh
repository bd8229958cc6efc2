#!/bin/bash
# Round-6 GPU steps: every GPU step under its own time limit, chained so that a crash or a
# timeout ends the call (no retries).  Usage: tools/r6_gpu.sh STEP...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r6
mkdir -p "$OUT"
( while sleep 30; do date +%T >> "$OUT/heartbeat"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() {  # run NAME SECONDS CMD...: log to $OUT/NAME.log; stop on a signal / timeout exit
    local name=$1 secs=$2; shift 2
    echo "== $name: $*" | tee -a "$OUT/steps.log"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
    tail -5 "$OUT/$name.log"
    if [ $rc -ge 124 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
    return 0
}
for step in "$@"; do
    case $step in
        parity1000) run parity1000 600 python -u tools/parity_1000.py --phase gpu ;;
        perturb) run perturb 600 python -u tools/parity_1000.py --phase perturb --record gpurun_out/r6/parity/dps_1000_steps.json ;;
        onestep) run onestep 300 python -u tools/parity_1000.py --phase onestep-gpu --case identity ;;
        bf16tests) run bf16_tests 900 python -u -m pytest tests/test_bf16_gpu.py -v --timeout 400 --timeout-method thread ;;
        bf16kern) run bf16_kern 600 python -u -m pytest tests/test_bf16_gpu.py -v --timeout 300 --timeout-method thread -k "conv3x3 or groupnorm or attention" ;;
        psldbf16) run psld_bf16 900 python -u tools/bench_psld.py --dtype bf16 --steps 3 --warmup 2 --cpu-baseline ;;
        psldbf16q) run psld_bf16 600 python -u tools/bench_psld.py --dtype bf16 --steps 3 --warmup 2 ;;
        psldbf16prof) run psld_bf16_prof 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof_psld_bf16" -o run -- python -u tools/bench_psld.py --dtype bf16 --steps 2 --warmup 1 ;;
        convab) run conv_ab_base 300 env SAMPLERS_HIP_LIB=samplers_amd/lib/variants/lib_${BASE:-norr}.so python -u tools/bench_conv_bf16.py
                run conv_ab_new 300 python -u tools/bench_conv_bf16.py ;;
        psldab) run psld_ab_base 600 env SAMPLERS_HIP_LIB=samplers_amd/lib/variants/lib_${BASE:-norr}.so python -u tools/bench_psld.py --dtype bf16 --steps 3 --warmup 2
                run psld_ab_new 600 python -u tools/bench_psld.py --dtype bf16 --steps 3 --warmup 2 ;;
        x6ab) run x6_desc_tests 300 env SAMPLERS_HIP_LIB=samplers_amd/lib/variants/lib_desc.so python -u -m pytest tests/test_gemm_x6_gpu.py -x -q --timeout 200 --timeout-method thread
              run x6_base 300 python -u tools/bench_gemm_x6.py
              run x6_desc 300 env SAMPLERS_HIP_LIB=samplers_amd/lib/variants/lib_desc.so python -u tools/bench_gemm_x6.py
              run x6_base2 300 python -u tools/bench_gemm_x6.py ;;
        resab) run psld_res_off 600 env SAMPLERS_AMD_BF16_RESNET=0 python -u tools/bench_psld.py --dtype bf16 --steps 3 --warmup 2
               run psld_res_on 600 python -u tools/bench_psld.py --dtype bf16 --steps 3 --warmup 2 ;;
        gnab) run gn_ab_base 300 env SAMPLERS_HIP_LIB=samplers_amd/lib/variants/lib_${BASE:-gnu1}.so python -u tools/bench_gn_bf16.py
              run gn_ab_new 300 python -u tools/bench_gn_bf16.py ;;
        gegluab) run psld_geglu_off 600 env SAMPLERS_AMD_BF16_GEGLU=0 python -u tools/bench_psld.py --dtype bf16 --steps 3 --warmup 2
                 run psld_geglu_on 600 python -u tools/bench_psld.py --dtype bf16 --steps 3 --warmup 2 ;;
        lnab) run psld_ln_off 600 env SAMPLERS_AMD_BF16_LN=0 SAMPLERS_AMD_BF16_GEGLU=0 python -u tools/bench_psld.py --dtype bf16 --steps 3 --warmup 2
              run psld_ln_on 600 python -u tools/bench_psld.py --dtype bf16 --steps 3 --warmup 2 ;;
        convexp7) run conv_exp7 300 env SAMPLERS_HIP_LIB=samplers_amd/lib/variants/lib_exp7.so python -u tools/bench_conv_bf16.py
                  run conv_base7 300 python -u tools/bench_conv_bf16.py ;;
        convexp8) run conv_exp8 300 env SAMPLERS_HIP_LIB=samplers_amd/lib/variants/lib_exp8.so python -u tools/bench_conv_bf16.py
                  run conv_base8 300 python -u tools/bench_conv_bf16.py ;;
        convexp9) run conv_exp9 300 env SAMPLERS_HIP_LIB=samplers_amd/lib/variants/lib_exp9.so python -u tools/bench_conv_bf16.py
                  run conv_base9 300 python -u tools/bench_conv_bf16.py ;;
        convexp10) run conv_exp10 300 env SAMPLERS_HIP_LIB=samplers_amd/lib/variants/lib_exp10.so python -u tools/bench_conv_bf16.py
                   run conv_base10 300 python -u tools/bench_conv_bf16.py ;;
        blkab) run psld_blk_off 600 env SAMPLERS_AMD_BF16_BLOCKED=0 python -u tools/bench_psld.py --dtype bf16 --steps 3 --warmup 2
               run psld_blk_on 600 python -u tools/bench_psld.py --dtype bf16 --steps 3 --warmup 2 ;;
        convbf16) run conv_bf16 300 python -u tools/bench_conv_bf16.py --miopen ;;
        convbf16sq) FILTER=k_conv3x3_bf16 NAME=convbf16 run conv_bf16_sq 600 tools/sq_pmc.sh tools/bench_conv_bf16.py --reps 3 --shapes sd ;;
        gputests) run gpu_tests 1100 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
done
