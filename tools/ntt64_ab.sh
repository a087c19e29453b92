#!/bin/bash
for round in 1 2; do
  for v in "$@"; do
    echo "$v r$round: $(FHE_AMD_LIB=abv/$v.so timeout -k 10 120 python tools/ntt_time.py 4096 400 ip 1152921504606830593 2>&1 | grep 'Q=' | tr '\n' ' ')" || exit 1
  done
done
