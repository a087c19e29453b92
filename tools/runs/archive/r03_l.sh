# round 3, GPU call L: 60-bit NTT with the first polynomial's layout-A stages ahead of the table barrier
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ntt.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03_l_ntt_tests.txt 2>&1 || { echo ntt-tests-failed; tail -20 gpurun_out/r03_l_ntt_tests.txt; exit 1; }
tail -2 gpurun_out/r03_l_ntt_tests.txt
timeout -k 10 400 bash tools/ntt64_ab.sh sol2 ntt_pre > gpurun_out/r03_l_ntt64_ab.txt 2>&1 || { echo ab-failed; cat gpurun_out/r03_l_ntt64_ab.txt; exit 1; }
cat gpurun_out/r03_l_ntt64_ab.txt
FHE_AMD_LIB=abv/ntt_pre.so timeout -k 10 120 python tools/ntt_time.py 4096 400 ip 134215681 2>&1 | grep Q=
