#!/bin/bash
# Round 4: K1w at 2^27 <= Q < 2^29 (GINX STD256 / STD256_3 with q = 2048; LMKCDEY STD256_3 / STD256_4) and
# 4 digits (STD256Q_4_LMKCDEY): parity against the 64-bit / A32 accumulator and the reference goldens, then
# the rates with K1w and on K5 A32 (FHE_HIP_N2K=0).
set -o pipefail
export FHE_SEGV_TRACE=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_paramsets.py -m gpu -k "n2k or std256" > gpurun_out/r04_qm2_tests.txt 2>&1 || { tail -c 6000 gpurun_out/r04_qm2_tests.txt; exit 1; }
tail -3 gpurun_out/r04_qm2_tests.txt
echo "FHE_HIP_N2K=1" >> gpurun_out/r04_qm2_bench.txt
timeout -k 10 200 python -u tools/bench_sets.py std256 std256_3 std256q std256_3_lmkcdey std256_4_lmkcdey std256q_4_lmkcdey >> gpurun_out/r04_qm2_bench.txt 2>&1 || exit 1
echo "FHE_HIP_N2K=0" >> gpurun_out/r04_qm2_bench.txt
FHE_HIP_N2K=0 timeout -k 10 200 python -u tools/bench_sets.py std256 std256_3 >> gpurun_out/r04_qm2_bench.txt 2>&1 || exit 1
cat gpurun_out/r04_qm2_bench.txt
