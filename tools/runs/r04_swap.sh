#!/bin/bash
# Round 4: K1w-LMKCDEY component-role swap (AUTO work split across the SIMDs), parity and A/B
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_paramsets.py -m gpu -k "n2k or std256q_3_lmkcdey" > gpurun_out/r04_swap_tests.txt 2>&1 || { tail -c 5000 gpurun_out/r04_swap_tests.txt; exit 1; }
tail -2 gpurun_out/r04_swap_tests.txt
o=gpurun_out/r04_swap_ab.txt; : > $o
for r in 1 2; do
  echo "swap=1 r$r" >> $o; timeout -k 10 120 python -u tools/bench_sets.py std256q_3_lmkcdey >> $o 2>&1 || exit 1
  echo "swap=0 r$r" >> $o; FHE_AMD_LIB=abv/swap0.so timeout -k 10 120 python -u tools/bench_sets.py std256q_3_lmkcdey >> $o 2>&1 || exit 1
done
cat $o
