# round 3, GPU call M: 32-bit NTT without the clamped prefetch when every wave has one polynomial
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ntt.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03_m_ntt_tests.txt 2>&1 || { echo ntt-tests-failed; tail -20 gpurun_out/r03_m_ntt_tests.txt; exit 1; }
tail -2 gpurun_out/r03_m_ntt_tests.txt
for round in 1 2 3; do
  for v in ntt_pre ntt32pf; do
    echo "$v r$round: $(FHE_AMD_LIB=abv/$v.so timeout -k 10 120 python tools/ntt_time.py 4096 400 ip 134215681,1152921504606830593 2>&1 | grep 'Q=' | tr '\n' ' ')" || exit 1
  done
done | tee gpurun_out/r03_m_ntt_ab.txt
