# A/B of the GINX key-prefetch variants at config 3's batch (1024) and the bench batch (65536)
set -o pipefail
mkdir -p gpurun_out
bash tools/ab.sh ginx 1024 base l2pf pf3 pf4w1 > gpurun_out/ab_pf_1024.txt 2>&1 || { cat gpurun_out/ab_pf_1024.txt; exit 1; }
cat gpurun_out/ab_pf_1024.txt
bash tools/ab.sh ginx 65536 base l2pf pf3 > gpurun_out/ab_pf_65536.txt 2>&1 || { cat gpurun_out/ab_pf_65536.txt; exit 1; }
cat gpurun_out/ab_pf_65536.txt
echo "split (K1s ND=2, base lib) at 1024:"
FHE_HIP_GINX_KERNEL=split FHE_AMD_LIB=abv/base.so timeout -k 10 120 python tools/gate_time.py ginx 1024 2>&1 | grep "B=" || exit 1
