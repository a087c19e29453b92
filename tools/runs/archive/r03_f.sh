# round 3, GPU call F: 60-bit NTT occupancy A/B; the 32-bit wide accumulator (A32): parity on every
# parameter set, then throughput against the 64-bit policy
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_paramsets.py tests/test_large.py tests/test_gates.py tests/test_backend.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r03_f_tests.txt 2>&1; rc=$?
tail -15 gpurun_out/r03_f_tests.txt
[ $rc -eq 0 ] || exit $rc
for s in std256 std256q_4 std256_lmkcdey std256q_3_lmkcdey; do
  timeout -k 10 200 python -u tools/bench_sets.py $s 2>&1 | grep gates/s | sed 's/^/narrow /' || exit 1
  FHE_HIP_NARROW=0 timeout -k 10 200 python -u tools/bench_sets.py $s 2>&1 | grep gates/s | sed 's/^/wide64 /' || exit 1
done | tee gpurun_out/r03_f_bench_sets.txt
