#!/bin/bash
# Round 4: K1w-LMKCDEY with 2 (28-bit Q) and 4 digits (parity, FHE_HIP_N2K_EXT=1), the u32 key switch,
# their rates, then the final-B evidence run
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_paramsets.py -m gpu -k "n2k" > gpurun_out/r04_nd4_tests.txt 2>&1 || { tail -c 5000 gpurun_out/r04_nd4_tests.txt; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r04_nd4_tests.txt | tail -6
bash tools/runs/r04_ksw.sh || exit $?
o=gpurun_out/r04_ext_bench.txt; : > $o
echo "EXT=1 KS32W=1" >> $o; FHE_HIP_N2K_EXT=1 FHE_HIP_KS32W=1 timeout -k 10 300 python -u tools/bench_sets.py std256q_lmkcdey std256q_4_lmkcdey >> $o 2>&1 || exit 1
echo "EXT=1 KS32W=0" >> $o; FHE_HIP_N2K_EXT=1 timeout -k 10 300 python -u tools/bench_sets.py std256q_lmkcdey std256q_4_lmkcdey >> $o 2>&1 || exit 1
echo "default (EXT=0, KS32W=0)" >> $o; timeout -k 10 300 python -u tools/bench_sets.py std256q_lmkcdey std256q_4_lmkcdey >> $o 2>&1 || exit 1
cat $o
bash tools/runs/r04_final_b.sh
