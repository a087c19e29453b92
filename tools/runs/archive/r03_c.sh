# round 3, GPU call C: 60-bit NTT A/B timing + rocprof, LDS bank-conflict attribution by ablation
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 bash tools/ntt64_ab.sh sol lazy solcopy > gpurun_out/r03_c_ntt64_ab.txt 2>&1 || { echo ab-failed; cat gpurun_out/r03_c_ntt64_ab.txt; exit 1; }
cat gpurun_out/r03_c_ntt64_ab.txt
FHE_AMD_LIB=abv/sol.so timeout -k 10 120 python tools/ntt_time.py 4096 400 ip 134215681 2>&1 | grep Q=
bash tools/prof_stats.sh r03_ntt64 tools/ntt_time.py 4096 50 ip 1152921504606830593,134215681 || exit 1
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/r03_avail.txt 2>&1 || true
timeout -k 10 1500 bash tools/pmc_lds.sh 8192 base abl4 abl2 abl256 abl512 notwpre > gpurun_out/r03_c_pmc_lds.txt 2>&1 || { echo pmc-failed; tail -20 gpurun_out/r03_c_pmc_lds.txt; exit 1; }
cat gpurun_out/r03_c_pmc_lds.txt
echo all-done
