# (1) the 64-bit NTT with 16-wave workgroups and a tile per plane (abv/ntp.so): parity tests, then
#     interleaved timing vs the production build; (2) key-switch tile variants (tools/r03_ks_ab.sh)
set -o pipefail
mkdir -p gpurun_out
FHE_AMD_LIB=abv/ntp.so timeout -k 10 300 python -u -m pytest tests/test_ntt.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ntp_tests.txt 2>&1 || { tail -30 gpurun_out/ntp_tests.txt; exit 1; }
tail -1 gpurun_out/ntp_tests.txt
bash tools/ntt64_ab.sh base ntp | tee gpurun_out/ntp_ab.txt || exit 1
bash tools/r03_ks_ab.sh
