#!/bin/bash
# round 6: K1m-4 with K1q's shared exchange area (FHE_M4_X128=1) vs per-wave planes, interleaved; then the LMKCDEY
# small-batch parity test on the x128 build
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r06_m4_x128_ab.txt
: > $out
for r in 1 2 3; do
  for v in base m4x; do
    echo -n "$v r$r: " >> $out
    FHE_AMD_LIB=abv/$v.so timeout -k 10 200 python -u tools/gate_time.py lmk 1 64 256 2>&1 | grep "^B=" | \
      sed 's/ms\/batch.*correct=/ms /' | tr '\n' ' ' >> $out || exit 1
    echo >> $out
  done
done
cat $out
FHE_AMD_LIB=abv/m4x.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gates.py -k "lmk" 2>&1 | tail -2
