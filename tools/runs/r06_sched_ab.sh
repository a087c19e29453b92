#!/bin/bash
# bootstrap.hip built with the AMDGPU max-ILP / max-memory-clause scheduling strategies vs the default:
# K1 (65,536 and 1024 gates), K1x (512), LMKCDEY op-list (16,384); two interleaved rounds
set -e
for round in 1 2; do
  for v in base bilp bmem; do
    echo -n "$v r$round: "
    FHE_AMD_LIB=abv/$v.so timeout -k 10 200 python tools/gate_time.py ginx 512 1024 65536 2>&1 | grep "B=" | sed 's/ms.batch.*correct=/ms /' | tr '\n' ' '
    FHE_AMD_LIB=abv/$v.so timeout -k 10 120 python tools/gate_time.py lmk 16384 2>&1 | grep "B=" | sed 's/ms.batch.*correct=/ms /' | tr '\n' ' '; echo
  done
done
