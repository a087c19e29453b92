#!/bin/bash
# Round 4: rocprofv3 kernel stats of the K1w rows added late in the round (per-kernel durations behind
# profiles/r04_k1w_*_bench.txt)
set -o pipefail
bash tools/prof_stats.sh r04_k1w_rows tools/bench_sets.py std256 std256_4 std256q_3 std256_3_lmkcdey std256q_4_lmkcdey > gpurun_out/r04_prof_k1w.txt 2>&1 || { cat gpurun_out/r04_prof_k1w.txt; exit 1; }
cat gpurun_out/r04_prof_k1w.txt
