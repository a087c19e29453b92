# round 3, GPU call I: issue / LDS / barrier counters of the A32 wide kernels (STD256 GINX, STD256_LMKCDEY)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in std256 std256_lmkcdey; do
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS \
      SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU --kernel-trace --output-format csv -d gpurun_out/pmc_narrow/$s -o run \
      -- python3 tools/bench_sets.py $s > gpurun_out/pmc_narrow_$s.log 2>&1 || { echo "pmc $s failed"; tail -5 gpurun_out/pmc_narrow_$s.log; exit 1; }
  python3 - gpurun_out/pmc_narrow/$s <<'PY'
import collections, csv, glob, sys
agg = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][:70]
        if "blind_rotate" in k:
            agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
for (k, c), v in sorted(agg.items()):
    print(f"{sys.argv[1].split('/')[-1]:16s} {k:70s} {c:22s} {v:.5g}")
PY
done | tee gpurun_out/r03_i_pmc_narrow.txt
