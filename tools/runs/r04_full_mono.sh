#!/bin/bash
# Round 4: K1w GINX with the full-resolution monomials (q = 2N: STD256_4): parity, then the rate with K1w
# and on K5 A32 (FHE_HIP_N2K=0)
set -o pipefail
export FHE_SEGV_TRACE=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_paramsets.py -m gpu -k "n2k and std256q_" > gpurun_out/r04_fm_tests.txt 2>&1 || { tail -c 6000 gpurun_out/r04_fm_tests.txt; exit 1; }
tail -3 gpurun_out/r04_fm_tests.txt
echo "FHE_HIP_N2K=1" >> gpurun_out/r04_fm_bench.txt
timeout -k 10 200 python -u tools/bench_sets.py std256q_3 std256q_4 >> gpurun_out/r04_fm_bench.txt 2>&1 || exit 1
echo "FHE_HIP_N2K=0" >> gpurun_out/r04_fm_bench.txt
FHE_HIP_N2K=0 timeout -k 10 200 python -u tools/bench_sets.py std256q_3 std256q_4 >> gpurun_out/r04_fm_bench.txt 2>&1 || exit 1
cat gpurun_out/r04_fm_bench.txt
