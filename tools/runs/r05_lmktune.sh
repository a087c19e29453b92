#!/bin/bash
# Round 5: LMKCDEY op-list kernel knobs re-measured on the round-5 kernel (waves per SIMD, key prefetch
# depths, twiddle preload, the first key chunk before the transforms), 65,536 gates, interleaved
set -o pipefail
export TMPDIR=/tmp
cp fhe_amd/libfhe_amd.so abv/base.so
o=gpurun_out/r05_lmktune_ab.txt; : > $o
for r in 1 2; do for v in base early w3 kpf2 akpf2 pre0; do
  FHE_AMD_LIB=abv/$v.so timeout -k 10 300 python tools/gate_time.py lmk 65536 > gpurun_out/r05_lmktune_t.txt 2>&1 || { tail -5 gpurun_out/r05_lmktune_t.txt; exit 1; }
  echo "$v r$r: $(tr '\n' ' ' < gpurun_out/r05_lmktune_t.txt)" >> $o
done; done
cat $o
