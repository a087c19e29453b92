# round 3, GPU call B: the 60-bit NTT (Sol60 butterflies, new data path): parity, then A/B timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ntt.py -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r03_b_ntt_tests.log 2>&1 || { echo tests-failed; tail -40 gpurun_out/r03_b_ntt_tests.log; exit 1; }
tail -3 gpurun_out/r03_b_ntt_tests.log
timeout -k 10 600 bash tools/ntt64_ab.sh sol lazy solcopy > gpurun_out/r03_b_ntt64_ab.txt 2>&1 || { echo ab-failed; cat gpurun_out/r03_b_ntt64_ab.txt; exit 1; }
cat gpurun_out/r03_b_ntt64_ab.txt
FHE_AMD_LIB=build/variants/sol.so timeout -k 10 120 python tools/ntt_time.py 4096 400 ip 134215681 2>&1 | grep Q=
echo all-done
