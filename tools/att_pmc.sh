set -o pipefail
mkdir -p gpurun_out/att
timeout -k 10 300 python -u tools/bench_attention.py > gpurun_out/att/attn.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/att/attn.log
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for c in FETCH_SIZE WRITE_SIZE; do
timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/att/pmc_$c -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/att/pmc_$c.log 2>&1 || exit $?
done
