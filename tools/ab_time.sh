#!/bin/bash
# timing-only A/B (ablation builds produce wrong results by design): method batch variants...
m=$1; b=$2; shift 2
for v in "$@"; do
  echo -n "$v: "; FHE_AMD_LIB=build/variants/$v.so timeout -k 10 120 python tools/gate_time.py $m $b 2>&1 | grep "B=" | sed 's/correct=.*//' || exit 1
done
