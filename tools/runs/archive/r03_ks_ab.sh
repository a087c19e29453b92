# key-switch tile variants: rocprofv3 kernel trace of tools/gate_time.py (GINX) at 65536 / 8192 / 1024
# gates, grouped by grid size
set -o pipefail
export TMPDIR=/tmp
for v in base ks512 ks512i2 ksi2; do
  echo "== $v"
  FHE_AMD_LIB=abv/$v.so bash tools/prof_stats.sh ks_$v tools/gate_time.py ginx 65536 8192 1024 > gpurun_out/ks_$v.txt 2>&1 || { cat gpurun_out/ks_$v.txt; exit 1; }
  grep -E "B=" gpurun_out/prof/ks_$v/log.txt
  python tools/trace_by_grid.py gpurun_out/prof/ks_$v/run_kernel_trace.csv | grep -E "keyswitch" || exit 1
done
