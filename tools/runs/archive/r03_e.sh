# round 3, GPU call E: 60-bit NTT occupancy / prefetch A/B and issue counters
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 bash tools/ntt64_ab.sh sol2 sol2w2 sol2w3 > gpurun_out/r03_e_ntt64_ab.txt 2>&1 || { echo ab-failed; cat gpurun_out/r03_e_ntt64_ab.txt; exit 1; }
cat gpurun_out/r03_e_ntt64_ab.txt
timeout -k 10 400 bash tools/pmc_ntt.sh sol sol2 sol2w2 > gpurun_out/r03_e_pmc_ntt.txt 2>&1 || { echo pmc-failed; tail -20 gpurun_out/r03_e_pmc_ntt.txt; exit 1; }
cat gpurun_out/r03_e_pmc_ntt.txt
