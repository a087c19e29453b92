# key-switch column tiles: 64 (production) vs 32 columns per workgroup (FHE_KS_COLS), and 32 columns
# with the 512-gate / two-values-of-i tiles from 8192 gates; per-launch times at 65536 / 16384 / 8192 /
# 1024 gates (rocprofv3, grouped by grid); parity of kc32w8 through the key-switch tests first
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
FHE_AMD_LIB=abv/kc32w8.so timeout -k 10 600 python -u -m pytest tests/test_gates.py tests/test_full.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/kc32w8_tests.txt 2>&1 || { tail -30 gpurun_out/kc32w8_tests.txt; exit 1; }
tail -1 gpurun_out/kc32w8_tests.txt
for v in kbase kc32 kc32w8; do
  FHE_AMD_LIB=abv/$v.so bash tools/prof_stats.sh kc_$v tools/gate_time.py ginx 65536 16384 8192 1024 > gpurun_out/kc_$v.txt 2>&1 || { cat gpurun_out/kc_$v.txt; exit 1; }
  echo "== $v"; grep -E "B=" gpurun_out/prof/kc_$v/log.txt
  python tools/trace_by_grid.py gpurun_out/prof/kc_$v/run_kernel_trace.csv | grep -E "keyswitch" || exit 1
done
