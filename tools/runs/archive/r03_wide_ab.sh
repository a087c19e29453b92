# the wide accumulator (bootstrap_wide.hip): LDS-only workgroup barriers (wlds) and, on top, the A32
# key prefetch per gadget level (wkpf) vs the production build (wbase); parity of the N = 2048 / wide
# sets with wkpf first
set -o pipefail
mkdir -p gpurun_out
FHE_AMD_LIB=abv/wkpf.so timeout -k 10 600 python -u -m pytest tests/test_paramsets.py tests/test_large.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/wkpf_tests.txt 2>&1 || { tail -30 gpurun_out/wkpf_tests.txt; exit 1; }
tail -1 gpurun_out/wkpf_tests.txt
for round in 1 2; do
  for v in wbase wlds wkpf; do
    FHE_AMD_LIB=abv/$v.so timeout -k 10 300 python tools/bench_sets.py std256 std256q std256q_4 std256_lmkcdey std256q_3_lmkcdey std192 2>&1 | grep "gates/s" | sed "s/^/$v r$round /" || exit 1
  done
done
