#!/bin/bash
# Round 5: cost of the sequential op emission in k_prep_lmk_w, by repeating it three times (FHE_PREP_REP=3)
set -o pipefail
export TMPDIR=/tmp
cp fhe_amd/libfhe_amd.so abv/base.so
o=gpurun_out/r05_emit_ab.txt; : > $o
for v in base emit3; do
  FHE_AMD_LIB=abv/$v.so timeout -k 10 300 bash tools/prof_stats.sh emit_$v tools/gate_time.py lmk 65536 > gpurun_out/r05_emit_$v.txt 2>&1 || { tail -5 gpurun_out/r05_emit_$v.txt; exit 1; }
  echo "== $v" >> $o; grep -i "prep_lmk\|blind_rotate_lmk\|gates/s" gpurun_out/r05_emit_$v.txt >> $o
done
cat $o
