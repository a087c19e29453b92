#!/bin/bash
# Round 4: the u32-sum tiled key switch (qKS 2^17 / 2^21 rows): parity vs the reference goldens, rates on/off
set -o pipefail
FHE_HIP_KS32W=1 timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_paramsets.py -m gpu -k "std192q_4 or std256q_4" > gpurun_out/r04_ksw_tests.txt 2>&1 || { tail -c 5000 gpurun_out/r04_ksw_tests.txt; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r04_ksw_tests.txt | tail -8
o=gpurun_out/r04_ksw_bench.txt; : > $o
echo "KS32W=1 (u32 sums)" >> $o; FHE_HIP_KS32W=1 timeout -k 10 300 python -u tools/bench_sets.py std192q_4 std256q_4 std256q_4_lmkcdey >> $o 2>&1 || exit 1
echo "KS32W=0" >> $o; FHE_HIP_KS32W=0 timeout -k 10 300 python -u tools/bench_sets.py std192q_4 std256q_4 std256q_4_lmkcdey >> $o 2>&1 || exit 1
cat $o
