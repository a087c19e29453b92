#!/bin/bash
# Round 5: the 4-digit K1w GINX form at Q < 2^27 without forward reductions (QM 3), parity then A/B vs QM 2
set -o pipefail
o=gpurun_out/r05_gpu_tests_qm3.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_paramsets.py tests/test_backend.py -m gpu -k "std256q_3 or std256q_4 or std256q" > $o 2>&1 || { tail -c 6000 $o; exit 1; }
tail -3 $o
cp fhe_amd/libfhe_amd.so abv/base.so
o=gpurun_out/r05_qm3_ab.txt; : > $o
for r in 1 2; do
  for v in base noqm3; do
    echo "== $v r$r" >> $o
    FHE_AMD_LIB=abv/$v.so timeout -k 10 300 python -u tools/bench_sets.py std256q_3 std256q_4 >> $o 2>&1 || { cat $o; exit 1; }
  done
done
cat $o
