#!/bin/bash
# Round 5: LMKCDEY op-list prep with the op emission through an LDS ring (FHE_PREP_RING): parity, then kernel times
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r05_gpu_tests_prep.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gates.py tests/test_full.py tests/test_fb.py tests/test_paramsets.py -m gpu -k "lmk or LMK or ap or AP" > $o 2>&1 || { tail -c 6000 $o; exit 1; }
tail -3 $o
cp fhe_amd/libfhe_amd.so abv/base.so
o=gpurun_out/r05_prep_ab.txt; : > $o
for v in base noring; do
  FHE_AMD_LIB=abv/$v.so timeout -k 10 300 bash tools/prof_stats.sh prep_$v tools/gate_time.py lmk 65536 > gpurun_out/r05_prep_$v.txt 2>&1 || { tail -5 gpurun_out/r05_prep_$v.txt; exit 1; }
  echo "== $v" >> $o; grep -i "prep_lmk\|blind_rotate_lmk" gpurun_out/r05_prep_$v.txt >> $o
done
cat $o
