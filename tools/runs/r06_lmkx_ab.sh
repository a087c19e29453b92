#!/bin/bash
# round 6: K1m's two-digit form (FHE_HIP_LMK_KERNEL=split) vs K1 LMK (wave) on STD128_LMKCDEY gate batches around
# the switch-over (x_batch_ = 512), interleaved rounds
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r06_lmkx_ab.txt
: > $out
for r in 1 2; do
  for k in split wave; do
    echo -n "$k r$r: " >> $out
    FHE_HIP_LMK_KERNEL=$k timeout -k 10 200 python -u tools/gate_time.py lmk 256 512 640 768 1024 2048 2>&1 | grep "^B=" | \
      sed 's/ms\/batch.*correct=/ms /' | tr '\n' ' ' >> $out || exit 1
    echo >> $out
  done
done
cat $out
