#!/bin/bash
# Round 5: T9 (first-stage product table) in the split and N = 2048 kernels (K1s, K1m, K1w): parity, then A/B
set -o pipefail
o=gpurun_out/r05_gpu_tests_t9w.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_paramsets.py -m gpu > $o 2>&1 || { tail -c 6000 $o; exit 1; }
tail -3 $o
cp fhe_amd/libfhe_amd.so abv/base.so
o=gpurun_out/r05_t9w_ab.txt; : > $o
for r in 1 2; do
  for v in base not9; do
    echo "== $v r$r" >> $o
    FHE_AMD_LIB=abv/$v.so timeout -k 10 400 python -u tools/bench_sets.py std256q std256q_3 std256_4 std256q_3_lmkcdey std128_3 std128_4_lmkcdey >> $o 2>&1 || { cat $o; exit 1; }
  done
done
cat $o
