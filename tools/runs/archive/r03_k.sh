# round 3, GPU call K: A32 gate kernel at 6 waves per SIMD (monomial table through the caches) vs 4
set -o pipefail
mkdir -p gpurun_out
for v in gcur g6; do
  for s in std256 std256q_4 std256q; do
    FHE_AMD_LIB=abv/$v.so timeout -k 10 200 python -u tools/bench_sets.py $s 2>&1 | grep gates/s | sed "s/^/$v /" || exit 1
  done
done | tee gpurun_out/r03_k_bench_sets.txt
