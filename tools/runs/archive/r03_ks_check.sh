# the key switch's tile shape by batch size: GPU tests, the bench line, per-launch key-switch times
# at 65536 / 32768 / 16384 / 8192 / 1024 gates for the build's threshold (32768), 16384 and "never";
# then the NTT wave-priority variants (abv/pr2, abv/pr4) vs abv/base
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
start=$(date +%s)
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r03_gputest_ks.txt 2>&1 || { echo pytest-failed; tail -30 gpurun_out/r03_gputest_ks.txt; exit 1; }
echo "pytest wall $(( $(date +%s) - start )) s"; tail -1 gpurun_out/r03_gputest_ks.txt
timeout -k 10 500 python bench.py > gpurun_out/r03_bench_ks.json 2> gpurun_out/r03_bench_ks.err || { echo bench-failed; tail -5 gpurun_out/r03_bench_ks.err; exit 1; }
cut -c1-300 gpurun_out/r03_bench_ks.json
for v in base ksw16 ksnever; do
  FHE_AMD_LIB=abv/$v.so bash tools/prof_stats.sh ksn_$v tools/gate_time.py ginx 65536 32768 16384 8192 1024 > gpurun_out/ksn_$v.txt 2>&1 || { cat gpurun_out/ksn_$v.txt; exit 1; }
  echo "== $v"; grep -E "B=" gpurun_out/prof/ksn_$v/log.txt
  python tools/trace_by_grid.py gpurun_out/prof/ksn_$v/run_kernel_trace.csv | grep -E "keyswitch" || exit 1
done
bash tools/ntt64_ab.sh base pr2 pr4 | tee gpurun_out/prio_ab.txt || exit 1
for v in base pr2 pr4; do
  echo "$v 32-bit: $(FHE_AMD_LIB=abv/$v.so timeout -k 10 120 python tools/ntt_time.py 4096 400 ip 134215681 2>&1 | grep 'Q=' | tr '\n' ' ')" || exit 1
done
