#!/bin/bash
# round 6: K1q's exchange with the four words of a slot side by side (FHE_Q_X128=1: one ds_read_b128) vs three
# b32 plane reads, interleaved; then K1q's parity tests on the x128 build
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r06_k1q_x128_ab.txt
: > $out
for r in 1 2 3; do
  for v in base x128; do
    echo -n "$v r$r: " >> $out
    FHE_AMD_LIB=abv/$v.so timeout -k 10 200 python -u tools/gate_time.py ginx 1 64 256 2>&1 | grep "^B=" | \
      sed 's/ms\/batch.*correct=/ms /' | tr '\n' ' ' >> $out || exit 1
    echo >> $out
  done
done
cat $out
FHE_AMD_LIB=abv/x128.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gates.py -k "qsplit or k1x" 2>&1 | tail -2
