#!/bin/bash
# Round 4: bisect the std192_lmkcdey null-accumulator failure, second step
set -o pipefail
run() {
  local name=$1; shift
  env "$@" > gpurun_out/$name.txt 2>&1; local rc=$?
  grep -E "PASSED|FAILED|passed|failed" gpurun_out/$name.txt | tail -8
  if [ $rc -gt 1 ]; then echo "stop: $name rc=$rc"; exit $rc; fi
}
T="timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_backend.py -m gpu"
echo "== keyswitch then null"; run r04_n3_a FHE_HIP_KS32=1 $T -k "std192_lmkcdey and (keyswitch or null)"
echo "== batch callers then null"; run r04_n3_b FHE_HIP_KS32=1 $T -k "std192_lmkcdey and (callers or null)"
echo "== all but keyswitch"; run r04_n3_c FHE_HIP_KS32=1 $T -k "std192_lmkcdey and not keyswitch"
echo "== all but callers"; run r04_n3_d FHE_HIP_KS32=1 $T -k "std192_lmkcdey and not callers"
echo "== lmkcdey (N = 1024) sequence"; run r04_n3_e FHE_HIP_KS32=1 $T -k "lmkcdey and not std192 and not std128_4"
echo "== std128_4_lmkcdey sequence"; run r04_n3_f FHE_HIP_KS32=1 $T -k "std128_4_lmkcdey"
