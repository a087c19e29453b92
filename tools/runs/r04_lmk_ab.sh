#!/bin/bash
# Round 4: LMKCDEY op-list kernel key-latency variants (abv/*.so), interleaved, 65,536 gates.
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do
  for v in "$@"; do
    echo -n "$v r$round: "
    FHE_AMD_LIB=abv/$v.so timeout -k 10 150 python tools/gate_time.py lmk 65536 2>&1 | grep "B=" || exit 1
  done
done
