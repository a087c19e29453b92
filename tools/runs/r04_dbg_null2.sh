#!/bin/bash
# Round 4: which earlier std192_lmkcdey backend test breaks the null-accumulator one
set -o pipefail
run() {
  local name=$1; shift
  env "$@" > gpurun_out/$name.txt 2>&1; local rc=$?
  grep -E "PASSED|FAILED|passed|failed" gpurun_out/$name.txt | tail -8
  if [ $rc -gt 1 ]; then echo "stop: $name rc=$rc"; exit $rc; fi
}
T="timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_backend.py -m gpu"
echo "== KS32=0 sequence"; run r04_n2_a FHE_HIP_KS32=0 $T -k "std192_lmkcdey"
echo "== KS32=1 sequence"; run r04_n2_b FHE_HIP_KS32=1 $T -k "std192_lmkcdey"
echo "== gate batch then null"; run r04_n2_c FHE_HIP_KS32=1 $T -k "std192_lmkcdey and (gate_batch or null)"
echo "== blind rotate then null"; run r04_n2_d FHE_HIP_KS32=1 $T -k "std192_lmkcdey and (blind_rotate or null)"
echo "== external product then null"; run r04_n2_e FHE_HIP_KS32=1 $T -k "std192_lmkcdey and (external or null)"
echo "== std192 (GINX) sequence"; run r04_n2_f FHE_HIP_KS32=1 $T -k "std192 and not lmkcdey"
