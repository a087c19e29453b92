#!/bin/bash
# Round 5: K1w GINX at one wave per SIMD (no scratch spills) vs two (spills), interleaved on one box
set -o pipefail
o=gpurun_out/r05_n2k_onewave.txt; : > $o
for r in 1 2; do
  for v in base n2kw1 n2kw3; do
    lib=fhe_amd/libfhe_amd.so; [ $v != base ] && lib=abv/$v.so
    echo "== $v r$r" >> $o
    FHE_AMD_LIB=$lib timeout -k 10 300 python -u tools/bench_sets.py std256q_3 std256q_4 std256_4 std256_3 std256q >> $o 2>&1 || { cat $o; exit 1; }
  done
done
cat $o
