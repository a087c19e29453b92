#!/bin/bash
# round 6: K1x's launch attributes for two-gate workgroups (waves_per_eu attribute vs launch-bounds minimum
# blocks), interleaved, device-resident gate batches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r06_k1x_lb_ab.txt
: > $out
for r in 1 2; do
  for v in base xlb1; do
    echo -n "$v r$r: " >> $out
    FHE_AMD_LIB=abv/$v.so timeout -k 10 200 python -u tools/gate_time.py ginx 1 64 256 257 512 2>&1 | grep "^B=" | \
      sed 's/ms\/batch.*correct=/ms /' | tr '\n' ' ' >> $out || exit 1
    echo >> $out
  done
done
cat $out
