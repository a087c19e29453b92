# the 60-bit NTT with phased loads (FHE_NTT64_PHASE): parity, then interleaved timing vs production
set -o pipefail
mkdir -p gpurun_out
FHE_AMD_LIB=abv/nphase.so timeout -k 10 300 python -u -m pytest tests/test_ntt.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/nphase_tests.txt 2>&1 || { tail -30 gpurun_out/nphase_tests.txt; exit 1; }
tail -1 gpurun_out/nphase_tests.txt
for round in 1 2 3; do
  for v in nbase nphase; do
    echo "$v r$round: $(FHE_AMD_LIB=abv/$v.so timeout -k 10 120 python tools/ntt_time.py 4096 400 ip 1152921504606830593 2>&1 | grep 'Q=' | tr '\n' ' ')" || exit 1
  done
done
