#!/bin/bash
# Round 4: the 32-bit tiled key switch on the 64-bit-path sets (ks32_) and K1w's LMKCDEY form (lmk2k):
# parity over every parameter set and the seam, then rates.
set -o pipefail
export FHE_SEGV_TRACE=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_paramsets.py -m gpu -k "n2k" > gpurun_out/r04_lmk2k_tests.txt 2>&1 || { tail -c 6000 gpurun_out/r04_lmk2k_tests.txt; exit 1; }
tail -3 gpurun_out/r04_lmk2k_tests.txt
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_paramsets.py tests/test_backend.py -m gpu > gpurun_out/r04_ks32_tests.txt 2>&1 || { tail -c 6000 gpurun_out/r04_ks32_tests.txt; exit 1; }
tail -3 gpurun_out/r04_ks32_tests.txt
o=gpurun_out/r04_ks32_bench.txt; : > $o
echo "default (K1w / lmk2k, KS32)" >> $o; timeout -k 10 200 python -u tools/bench_sets.py std256q std256q_3_lmkcdey std192 std256 >> $o 2>&1 || exit 1
echo "FHE_HIP_KS32=0" >> $o; FHE_HIP_KS32=0 timeout -k 10 200 python -u tools/bench_sets.py std256q std256q_3_lmkcdey std192 std256 >> $o 2>&1 || exit 1
echo "FHE_HIP_N2K=0 FHE_HIP_KS32=0" >> $o; FHE_HIP_N2K=0 FHE_HIP_KS32=0 timeout -k 10 200 python -u tools/bench_sets.py std256q_3_lmkcdey >> $o 2>&1 || exit 1
echo "A64: FHE_HIP_N2K=0 FHE_HIP_KS32=0 FHE_HIP_NARROW=0" >> $o; FHE_HIP_N2K=0 FHE_HIP_KS32=0 FHE_HIP_NARROW=0 timeout -k 10 200 python -u tools/bench_sets.py std256q_3_lmkcdey >> $o 2>&1 || exit 1
cat $o
