#!/bin/bash
# Round 5: the first forward stage's digit x twiddle products from an LDS table (T9): A/B, then the whole GPU suite
set -o pipefail
cp fhe_amd/libfhe_amd.so abv/base.so
o=gpurun_out/r05_t9_ab.txt; : > $o
for r in 1 2; do
  for v in base not9; do
    for m in ginx lmk; do
      echo -n "$v $m r$r: " >> $o
      FHE_AMD_LIB=abv/$v.so timeout -k 10 180 python tools/gate_time.py $m 1024 65536 2>&1 | grep "B=" | tr '\n' ' ' >> $o || { cat $o; exit 1; }
      echo >> $o
    done
  done
done
cat $o
o=gpurun_out/r05_gpu_tests_t9.txt
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $o 2>&1 || { tail -c 8000 $o; exit 1; }
tail -3 $o
