#!/bin/bash
# Round 4: K1w key prefetch on/off (abv/kpf0.so: FHE_N2K_KPF=0), interleaved, and the A64 / A32 baselines on STD256Q.
set -o pipefail
o=gpurun_out/r04_n2k_ab.txt; : > $o
for r in 1 2; do
  echo "K1w KPF=1 r$r" >> $o; timeout -k 10 120 python -u tools/bench_sets.py std256q >> $o 2>&1 || exit 1
  echo "K1w KPF=0 r$r" >> $o; FHE_AMD_LIB=abv/kpf0.so timeout -k 10 120 python -u tools/bench_sets.py std256q >> $o 2>&1 || exit 1
done
echo "A32 (FHE_HIP_N2K=0)" >> $o; FHE_HIP_N2K=0 timeout -k 10 120 python -u tools/bench_sets.py std256q >> $o 2>&1 || exit 1
echo "A64 (FHE_HIP_N2K=0 FHE_HIP_NARROW=0)" >> $o; FHE_HIP_N2K=0 FHE_HIP_NARROW=0 timeout -k 10 200 python -u tools/bench_sets.py std256q >> $o 2>&1 || exit 1
cat $o
