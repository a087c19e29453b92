#!/bin/bash
# Round 5: LMKCDEY op-list prep with lane-parallel emission offsets: parity, then kernel times vs the sequential emission
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r05_gpu_tests_emitpar.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gates.py tests/test_full.py tests/test_fb.py tests/test_paramsets.py tests/test_mixed.py -m gpu -k "lmk or LMK or ap or AP or std256q" > $o 2>&1 || { tail -c 6000 $o; exit 1; }
tail -3 $o
cp fhe_amd/libfhe_amd.so abv/base.so
o=gpurun_out/r05_emitpar_ab.txt; : > $o
for v in base old; do
  FHE_AMD_LIB=abv/$v.so timeout -k 10 300 bash tools/prof_stats.sh emitpar_$v tools/gate_time.py lmk 65536 > gpurun_out/r05_emitpar_$v.txt 2>&1 || { tail -5 gpurun_out/r05_emitpar_$v.txt; exit 1; }
  echo "== $v" >> $o; grep -i "prep_lmk\|blind_rotate_lmk\|gates/s" gpurun_out/r05_emitpar_$v.txt >> $o
done
cat $o
