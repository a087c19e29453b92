#!/bin/bash
# Round 5: the first forward stage's digit products from an LDS table (FHE_DT1): parity, then K1 times
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r05_gpu_tests_dt1.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gates.py tests/test_full.py tests/test_backend.py tests/test_paramsets.py -m gpu -k "not lmk and not LMK" > $o 2>&1 || { tail -c 6000 $o; exit 1; }
tail -3 $o
cp fhe_amd/libfhe_amd.so abv/base.so
o=gpurun_out/r05_dt1_ab.txt; : > $o
for r in 1 2; do for v in base nodt; do
  FHE_AMD_LIB=abv/$v.so timeout -k 10 300 python tools/gate_time.py ginx 1024 65536 > gpurun_out/r05_dt1_t.txt 2>&1 || { tail -5 gpurun_out/r05_dt1_t.txt; exit 1; }
  echo "$v r$r: $(tr '\n' ' ' < gpurun_out/r05_dt1_t.txt)" >> $o
done; done
cat $o
