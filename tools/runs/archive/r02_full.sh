set -o pipefail
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_gputest_all.log 2>&1 || { echo pytest-failed; tail -20 gpurun_out/r02_gputest_all.log; exit 1; }
tail -2 gpurun_out/r02_gputest_all.log
timeout -k 10 300 python bench.py > gpurun_out/r02_bench.json 2> gpurun_out/r02_bench.err || { echo bench-failed; exit 1; }
bash tools/prof_stats.sh r02_bench bench.py --no-cpu-baseline || exit 1
bash tools/pmc_run.sh 65536 || exit 1
echo all-done
