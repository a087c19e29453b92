#!/bin/bash
# Round 4: the std192_lmkcdey null-accumulator failure with the 32-bit key switch off / on, then the rest of
# the backend suite and the N = 2048 rates.
set -o pipefail
run() {  # name, env..., pytest args: stop on anything but pass / test failure
  local name=$1; shift
  env "$@" > gpurun_out/$name.txt 2>&1; local rc=$?
  tail -4 gpurun_out/$name.txt
  if [ $rc -gt 1 ]; then echo "stop: $name rc=$rc"; exit $rc; fi
}
T="timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_backend.py -m gpu"
run r04_null_ks0 FHE_HIP_KS32=0 $T -k "null_accumulators and std192_lmkcdey"
run r04_null_ks1 FHE_HIP_KS32=1 $T -k "null_accumulators and std192_lmkcdey"
run r04_null_all FHE_HIP_KS32=1 $T -k "std192_lmkcdey"
o=gpurun_out/r04_ks32_bench.txt; : > $o
echo "default (K1w / lmk2k, KS32)" >> $o; timeout -k 10 200 python -u tools/bench_sets.py std256q std256q_3_lmkcdey std192 std256 >> $o 2>&1 || exit 1
echo "FHE_HIP_KS32=0" >> $o; FHE_HIP_KS32=0 timeout -k 10 200 python -u tools/bench_sets.py std256q std256q_3_lmkcdey std192 std256 >> $o 2>&1 || exit 1
echo "FHE_HIP_N2K=0 FHE_HIP_KS32=0" >> $o; FHE_HIP_N2K=0 FHE_HIP_KS32=0 timeout -k 10 200 python -u tools/bench_sets.py std256q_3_lmkcdey >> $o 2>&1 || exit 1
echo "A64: FHE_HIP_N2K=0 FHE_HIP_KS32=0 FHE_HIP_NARROW=0" >> $o; FHE_HIP_N2K=0 FHE_HIP_KS32=0 FHE_HIP_NARROW=0 timeout -k 10 200 python -u tools/bench_sets.py std256q_3_lmkcdey >> $o 2>&1 || exit 1
cat $o
