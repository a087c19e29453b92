#!/bin/bash
# per-kernel rocprof stats of tools/gate_time.py for each library variant: tools/ks_prof.sh B variants...
b=$1; shift
for v in "$@"; do
  echo "== $v"
  FHE_AMD_LIB=build/variants/$v.so tools/prof_stats.sh ks_$v tools/gate_time.py ginx $b | grep -E "keyswitch|blind_rotate" || exit 1
done
