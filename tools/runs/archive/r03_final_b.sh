# round-3 final check, part B: the 2-rank rehearsal, the default bench line, rocprofv3 stats of the bench, PMC traffic passes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
FHE_BENCH_DEVICE_MAP=0,0 FHE_BENCH_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 2 --steps 3 --warmup 1 \
    --no-cpu-baseline > gpurun_out/r03_bench_rehearsal_w2.json 2> gpurun_out/r03_bench_rehearsal_w2.err || { echo rehearsal-failed; tail -20 gpurun_out/r03_bench_rehearsal_w2.err; exit 1; }
cat gpurun_out/r03_bench_rehearsal_w2.json
timeout -k 10 500 python bench.py > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err || { echo bench-failed; tail -5 gpurun_out/r03_bench.err; exit 1; }
cat gpurun_out/r03_bench.json
bash tools/prof_stats.sh r03_bench bench.py --no-cpu-baseline || exit 1
bash tools/pmc_run.sh 65536 || exit 1
echo part-b-done
