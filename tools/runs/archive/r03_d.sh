# round 3, GPU call D: VALU rates of the 64-bit ops, Sol60 NTT rewrite A/B + parity
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./abv/ubench > gpurun_out/r03_d_ubench.txt 2>&1 || { echo ubench-failed; cat gpurun_out/r03_d_ubench.txt; exit 1; }
cat gpurun_out/r03_d_ubench.txt
timeout -k 10 600 bash tools/ntt64_ab.sh sol sol2 sol2copy > gpurun_out/r03_d_ntt64_ab.txt 2>&1 || { echo ab-failed; cat gpurun_out/r03_d_ntt64_ab.txt; exit 1; }
cat gpurun_out/r03_d_ntt64_ab.txt
timeout -k 10 300 python -u -m pytest tests/test_ntt.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03_d_ntt_tests.txt 2>&1; rc=$?
tail -5 gpurun_out/r03_d_ntt_tests.txt
exit $rc
