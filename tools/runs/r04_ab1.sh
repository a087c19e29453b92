#!/bin/bash
# Round 4: LMKCDEY op-list kernel occupancy variants (opq: per-op opaque lane addressing, 194 VGPRs;
# opq3: the same at 3 waves per SIMD) and the XCD-aware key-switch tile order (ksx), interleaved.
set -o pipefail
for round in 1 2; do
  for v in base opq opq3; do
    echo -n "lmk $v r$round: "
    FHE_AMD_LIB=abv/$v.so timeout -k 10 150 python tools/gate_time.py lmk 65536 2>&1 | grep "B=" || exit 1
  done
  for v in base ksx; do
    for B in 65536 16384; do
      echo -n "ks $v r$round: "
      FHE_AMD_LIB=abv/$v.so timeout -k 10 150 python tools/ks_time.py $B 20 2>&1 | grep "B=" || exit 1
    done
  done
done
