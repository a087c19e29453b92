#!/bin/bash
# Round 5: LMKCDEY automorphism digits by v_permlane32_swap (A/B vs the LDS pass), K1 at one wave per EU (1024 gates)
set -o pipefail
o=gpurun_out/r05_gpu_tests_lmkswap.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu -k "lmk or LMK" > $o 2>&1 || { tail -c 6000 $o; exit 1; }
tail -3 $o
cp fhe_amd/libfhe_amd.so abv/base.so
o=gpurun_out/r05_lmkswap_ab.txt; : > $o
for r in 1 2; do
  for v in base noswap; do
    echo -n "$v lmk r$r: " >> $o
    FHE_AMD_LIB=abv/$v.so timeout -k 10 180 python tools/gate_time.py lmk 1024 65536 2>&1 | grep "B=" | tr '\n' ' ' >> $o || { cat $o; exit 1; }
    echo >> $o
  done
  for v in base wpe1; do
    echo -n "$v ginx r$r: " >> $o
    FHE_AMD_LIB=abv/$v.so timeout -k 10 180 python tools/gate_time.py ginx 1024 2>&1 | grep "B=" | tr '\n' ' ' >> $o || { cat $o; exit 1; }
    echo >> $o
  done
done
cat $o
