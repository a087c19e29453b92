#!/bin/bash
# Time each variant (interleaved rounds) with tools/gate_time.py; args: method batch variants...
m=$1; b=$2; shift 2
for round in 1 2; do
  for v in "$@"; do
    echo -n "$v r$round: "; FHE_AMD_LIB=abv/$v.so timeout -k 10 120 python tools/gate_time.py $m $b 2>&1 | grep "B=" || exit 1
  done
done
