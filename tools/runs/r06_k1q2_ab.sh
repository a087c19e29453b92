#!/bin/bash
# round 6: K1q with single-buffered planes (two gates per CU) vs K1x for 257..512 gates (FHE_HIP_Q_BATCH=512 vs
# the default 256), interleaved; then the K1q parity tests (the pinned 1027-gate batch runs the single-buffered form)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r06_k1q2_ab.txt
: > $out
for r in 1 2; do
  for v in 512 256; do
    echo -n "qbatch=$v r$r: " >> $out
    FHE_HIP_Q_BATCH=$v timeout -k 10 200 python -u tools/gate_time.py ginx 256 384 512 2>&1 | grep "^B=" | \
      sed 's/ms\/batch.*correct=/ms /' | tr '\n' ' ' >> $out || exit 1
    echo >> $out
  done
done
cat $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gates.py -k "qsplit or k1x" 2>&1 | tail -2
