#!/bin/bash
# Round 5: K1 key chunks through buffer descriptors (scalar chunk offsets) vs 64-bit VGPR addresses
set -o pipefail
o=gpurun_out/r05_gpu_tests_kbuf.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gates.py tests/test_full.py tests/test_fb.py tests/test_backend.py tests/test_multi_gates.py -m gpu > $o 2>&1 || { tail -c 6000 $o; exit 1; }
tail -3 $o
cp fhe_amd/libfhe_amd.so abv/base.so
o=gpurun_out/r05_kbuf_ab.txt; : > $o
for r in 1 2 3; do
  for v in base nokbuf; do
    for m in ginx lmk; do
      echo -n "$v $m r$r: " >> $o
      FHE_AMD_LIB=abv/$v.so timeout -k 10 180 python tools/gate_time.py $m 1024 65536 2>&1 | grep "B=" | tr '\n' ' ' >> $o || { cat $o; exit 1; }
      echo >> $o
    done
  done
done
cat $o
