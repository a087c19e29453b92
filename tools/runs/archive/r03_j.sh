# round 3, GPU call J: wave-local syncs + LDS tables (gate kernel) + 32-bit decomposition in the wide accumulator's transforms: parity on every wide set, throughput
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_paramsets.py tests/test_large.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r03_j_tests.txt 2>&1; rc=$?
tail -3 gpurun_out/r03_j_tests.txt
[ $rc -eq 0 ] || exit $rc
for s in std256 std256q_4 std256_lmkcdey std256q_3_lmkcdey std192 std128q_4; do
  timeout -k 10 200 python -u tools/bench_sets.py $s 2>&1 | grep gates/s | sed "s/^/dec32 /" || exit 1
done | tee gpurun_out/r03_j_bench_sets.txt
