#!/bin/bash
# round 6: config 3 (1024 STD128 gates) on K1's ONE build (early key requests, one-wave register budget) vs the
# two-waves-per-SIMD build (FHE_HIP_K1_ONE=0), steady-state step times, interleaved
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r06_k1one_ab.txt
: > $out
for r in 1 2; do
  for v in 1 0; do
    echo -n "one=$v r$r: " >> $out
    FHE_HIP_K1_ONE=$v timeout -k 10 200 python -u tools/c3_ramp.py 120 2>&1 | grep "steps 40-80\|steps 80-" | tr '\n' ' ' >> $out || exit 1
    echo >> $out
  done
done
cat $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_full.py -k config3 2>&1 | tail -2
