# the op-list kernel's key prefetch (FHE_WIDE_KPF=2) at 6 and 5 waves per SIMD vs the gate-kernel-only
# prefetch build (wkpf); parity of the wide sets with wkpf2w5 first
set -o pipefail
mkdir -p gpurun_out
FHE_AMD_LIB=abv/wkpf2w5.so timeout -k 10 600 python -u -m pytest tests/test_paramsets.py tests/test_large.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/wkpf2_tests.txt 2>&1 || { tail -30 gpurun_out/wkpf2_tests.txt; exit 1; }
tail -1 gpurun_out/wkpf2_tests.txt
for round in 1 2; do
  for v in wkpf wkpf2 wkpf2w5; do
    FHE_AMD_LIB=abv/$v.so timeout -k 10 300 python tools/bench_sets.py std256_lmkcdey std256q_3_lmkcdey std192_lmkcdey 2>&1 | grep "gates/s" | sed "s/^/$v r$round /" || exit 1
  done
done
