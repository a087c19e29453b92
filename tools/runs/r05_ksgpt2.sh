#!/bin/bash
# Round 5: key-switch tiles of 1024 gates (2 gates per thread) vs 512 at 65,536 gates (timing), then parity
set -o pipefail
cp fhe_amd/libfhe_amd.so abv/base.so
o=gpurun_out/r05_ksgpt2_ab.txt; : > $o
for r in 1 2 3; do
  for v in base gpt2; do
    echo -n "$v r$r: " >> $o
    FHE_AMD_LIB=abv/$v.so timeout -k 10 180 python tools/gate_time.py ginx 16384 65536 2>&1 | grep "B=" | tr '\n' ' ' >> $o || { cat $o; exit 1; }
    echo >> $o
  done
done
cat $o
o=gpurun_out/r05_ksgpt2_prof.txt
FHE_AMD_LIB=abv/gpt2.so timeout -k 10 300 bash tools/prof_stats.sh ksgpt2 tools/gate_time.py ginx 65536 > $o 2>&1 || { tail -5 $o; exit 1; }
grep -i keyswitch $o
