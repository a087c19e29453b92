#!/bin/bash
# Round 5: K1 LMKCDEY time with the accumulator bound of centred keys (1.4Q / 1.2Q plans; timing only,
# the keys here are not centred)
set -o pipefail
export TMPDIR=/tmp
cp fhe_amd/libfhe_amd.so abv/base.so
o=gpurun_out/r05_acc14_ab.txt; : > $o
for r in 1 2; do for v in base acc14; do
  FHE_AMD_LIB=abv/$v.so timeout -k 10 300 bash tools/prof_stats.sh acc_${v}_$r tools/gate_time.py lmk 65536 > gpurun_out/r05_acc_$v.txt 2>&1 || { tail -5 gpurun_out/r05_acc_$v.txt; exit 1; }
  echo "== $v r$r" >> $o; grep -i "prep_lmk\|blind_rotate_lmk" gpurun_out/r05_acc_$v.txt >> $o
done; done
cat $o
