#!/bin/bash
# round-4 check, part B: smoke(), the 2-rank rehearsal, the default bench line, rocprofv3 stats of the
# bench, PMC traffic passes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_smoke.txt 2>&1 || { echo smoke-failed; tail -20 gpurun_out/r04_smoke.txt; exit 1; }
tail -1 gpurun_out/r04_smoke.txt
FHE_BENCH_DEVICE_MAP=0,0 FHE_BENCH_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 2 --steps 3 --warmup 1 \
    --no-cpu-baseline > gpurun_out/r04_bench_rehearsal_w2.json 2> gpurun_out/r04_bench_rehearsal_w2.err || { echo rehearsal-failed; tail -20 gpurun_out/r04_bench_rehearsal_w2.err; exit 1; }
cat gpurun_out/r04_bench_rehearsal_w2.json
timeout -k 10 500 python bench.py > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.err || { echo bench-failed; tail -5 gpurun_out/r04_bench.err; exit 1; }
cat gpurun_out/r04_bench.json
bash tools/prof_stats.sh r04_bench bench.py --no-cpu-baseline || exit 1
bash tools/pmc_run.sh 65536 || exit 1
python3 tools/pmc_traffic.py r04 65536 > gpurun_out/r04_pmc_traffic.json && cat gpurun_out/r04_pmc_traffic.json
echo part-b-done
