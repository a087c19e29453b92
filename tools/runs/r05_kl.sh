#!/bin/bash
# Round 5: K1 with LDS-staged keys (KL) at <= 1024 gates: timing A/B, then the whole GPU suite on the KL default
set -o pipefail
o=gpurun_out/r05_kl_ab.txt; : > $o
for r in 1 2; do
  for v in nokl kl klw1; do
    echo -n "$v r$r: " >> $o
    FHE_AMD_LIB=abv/$v.so timeout -k 10 180 python tools/gate_time.py ginx 256 1024 2048 2>&1 | grep "B=" | tr '\n' ' ' >> $o || { cat $o; exit 1; }
    echo >> $o
  done
done
cat $o
o=gpurun_out/r05_gpu_tests_kl.txt
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $o 2>&1 || { tail -c 8000 $o; exit 1; }
tail -3 $o
