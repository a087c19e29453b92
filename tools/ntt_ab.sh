#!/bin/bash
# Time NTT variants (interleaved rounds) for Q=134215681; args: count mode(ip|oop) variants...
c=$1; mode=$2; shift 2
for round in 1 2; do
  for v in "$@"; do
    echo "$v r$round: $(FHE_AMD_LIB=abv/$v.so timeout -k 10 120 python tools/ntt_time.py $c 400 $mode 134215681 2>&1 | grep 'Q=' | tr '\n' ' ')" || exit 1
  done
done
