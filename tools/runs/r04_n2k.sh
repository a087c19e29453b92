#!/bin/bash
# Round 4: the archive GPU test, the seam split, then K1w (N = 2048 GINX in registers) parity and rate on
# STD256Q.
set -o pipefail
export FHE_SEGV_TRACE=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_cereal.py -m gpu -k "context" > gpurun_out/r04_ctx.txt 2>&1 || { tail -c 6000 gpurun_out/r04_ctx.txt; exit 1; }
tail -3 gpurun_out/r04_ctx.txt
timeout -k 10 240 python -u tools/seam_split.py 2048 > gpurun_out/r04_seam_split.txt 2>&1 || { tail -c 3000 gpurun_out/r04_seam_split.txt; exit 1; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_paramsets.py -m gpu -k "n2k or std256q" > gpurun_out/r04_n2k_tests.txt 2>&1 || { tail -c 6000 gpurun_out/r04_n2k_tests.txt; exit 1; }
tail -3 gpurun_out/r04_n2k_tests.txt
for flag in 1 0; do
  echo "FHE_HIP_N2K=$flag" >> gpurun_out/r04_n2k_bench.txt; FHE_HIP_N2K=$flag timeout -k 10 170 python -u tools/bench_sets.py std256q >> gpurun_out/r04_n2k_bench.txt 2>&1 || exit 1
done
cat gpurun_out/r04_n2k_bench.txt
