#!/bin/bash
# Round 5: inverse plans with reductions before the transposes + forward bounds from the product (FM 2 / QM 2):
# the whole GPU suite, then A/B against the round-4 plans (old) and with the T9 table on (t9on)
set -o pipefail
o=gpurun_out/r05_gpu_tests_plans.txt
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $o 2>&1 || { tail -c 8000 $o; exit 1; }
tail -3 $o
cp fhe_amd/libfhe_amd.so abv/base.so
o=gpurun_out/r05_plans_ab.txt; : > $o
for r in 1 2; do
  for v in base old t9on; do
    for m in ginx lmk; do
      echo -n "$v $m r$r: " >> $o
      FHE_AMD_LIB=abv/$v.so timeout -k 10 180 python tools/gate_time.py $m 1024 65536 2>&1 | grep "B=" | tr '\n' ' ' >> $o || { cat $o; exit 1; }
      echo >> $o
    done
  done
done
for r in 1 2; do
  for v in base old; do
    echo "== $v r$r" >> $o
    FHE_AMD_LIB=abv/$v.so timeout -k 10 400 python -u tools/bench_sets.py std256q std256q_3 std256 std256_4 std256_3_lmkcdey std256q_3_lmkcdey std128_3 std128_4_lmkcdey >> $o 2>&1 || { cat $o; exit 1; }
  done
done
cat $o
