# round-3 final check: every GPU test, smoke(), the default bench line, rocprofv3 stats of the bench,
# PMC passes (FETCH/WRITE traffic, VALU busy), the 2-rank one-GPU rehearsal
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
start=$(date +%s)
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r03_gputest_all.txt 2>&1 || { echo pytest-failed; tail -30 gpurun_out/r03_gputest_all.txt; exit 1; }
echo "pytest wall $(( $(date +%s) - start )) s"; tail -1 gpurun_out/r03_gputest_all.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.txt 2>&1 || { echo smoke-failed; tail -20 gpurun_out/r03_smoke.txt; exit 1; }
tail -1 gpurun_out/r03_smoke.txt
timeout -k 10 500 python bench.py > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err || { echo bench-failed; tail -5 gpurun_out/r03_bench.err; exit 1; }
cut -c1-300 gpurun_out/r03_bench.json
bash tools/prof_stats.sh r03_bench bench.py --no-cpu-baseline || exit 1
bash tools/pmc_run.sh 65536 > gpurun_out/pmc_log.txt 2>&1 || { tail -5 gpurun_out/pmc_log.txt; exit 1; }
FHE_BENCH_DEVICE_MAP=0,0 FHE_BENCH_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 2 --steps 3 --warmup 1 \
    --no-cpu-baseline > gpurun_out/r03_bench_rehearsal_w2.json 2> gpurun_out/r03_bench_rehearsal_w2.err || { echo rehearsal-failed; tail -20 gpurun_out/r03_bench_rehearsal_w2.err; exit 1; }
cut -c1-200 gpurun_out/r03_bench_rehearsal_w2.json
echo final-done
