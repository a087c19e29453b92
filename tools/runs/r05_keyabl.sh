#!/bin/bash
# Round 5: how much of K1's time is key delivery? timing-only ablations (wrong results by design):
# ablk1 = keys from a 4 KB L1-resident block, ablk2 = no key loads
set -o pipefail
cp fhe_amd/libfhe_amd.so abv/base.so
o=gpurun_out/r05_keyabl.txt; : > $o
for r in 1 2; do
  for v in base ablk1 ablk2; do
    for m in ginx lmk; do
      echo -n "$v $m r$r: " >> $o
      FHE_AMD_LIB=abv/$v.so timeout -k 10 180 python tools/gate_time.py $m 1024 65536 2>&1 | grep "B=" | sed 's/correct=.*//' | tr '\n' ' ' >> $o || { cat $o; exit 1; }
      echo >> $o
    done
  done
done
cat $o
