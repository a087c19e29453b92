# round-2 final check, part B: rocprofv3 kernel-trace stats of the bench, PMC traffic passes
set -o pipefail
mkdir -p gpurun_out
bash tools/prof_stats.sh r02_bench bench.py --no-cpu-baseline || exit 1
bash tools/pmc_run.sh 65536 || exit 1
echo part-b-done
