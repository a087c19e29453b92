# round 3, GPU call H: the 32-bit wide accumulator with Harvey-lazy NTTs at 4 vs 6 waves per SIMD
set -o pipefail
mkdir -p gpurun_out
for v in nw4 nw6; do
  for s in std256 std256q_4 std256_lmkcdey std256q_3_lmkcdey; do
    FHE_AMD_LIB=abv/$v.so timeout -k 10 200 python -u tools/bench_sets.py $s 2>&1 | grep gates/s | sed "s/^/$v /" || exit 1
  done
done | tee gpurun_out/r03_h_bench_sets.txt
