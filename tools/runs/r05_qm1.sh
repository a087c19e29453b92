#!/bin/bash
# Round 5: K1w-LMKCDEY at 2^27 <= Q < 2^28 (QM 1) without its forward reduction: parity, then A/B vs round-4 plans
set -o pipefail
o=gpurun_out/r05_gpu_tests_qm1.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_paramsets.py tests/test_backend.py tests/test_mixed.py -m gpu -k "std256q_lmkcdey or std256q" > $o 2>&1 || { tail -c 6000 $o; exit 1; }
tail -3 $o
cp fhe_amd/libfhe_amd.so abv/base.so
o=gpurun_out/r05_qm1_ab.txt; : > $o
for r in 1 2; do
  for v in base old; do
    echo "== $v r$r" >> $o
    FHE_AMD_LIB=abv/$v.so timeout -k 10 300 python -u tools/bench_sets.py std256q_lmkcdey >> $o 2>&1 || { cat $o; exit 1; }
  done
done
cat $o
