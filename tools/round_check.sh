#!/bin/bash
# Full round check on one GPU: tests, smoke, benches (DPS inpaint + blur, PSLD, ReSample),
# rocprofv3 kernel stats of the headline bench, PMC traffic passes.  Output: gpurun_out/rc/
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rc
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench_inpaint.json 2> $O/bench_inpaint.err
timeout -k 10 300 python bench.py --config blur --no-cpu-baseline > $O/bench_blur.json 2> $O/bench_blur.err
timeout -k 10 400 python -u tools/bench_psld.py --warmup 2 > $O/bench_psld.json 2> $O/bench_psld.err
timeout -k 10 400 python -u tools/bench_resample.py --steps 4 > $O/bench_resample.json 2> $O/bench_resample.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $R/bench.py --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/prof.log
for c in FETCH_SIZE WRITE_SIZE; do
  d=$O/pmc_$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  mkdir -p $d
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $d -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $d.log 2>&1
done
