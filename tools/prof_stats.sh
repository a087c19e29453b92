#!/bin/bash
# rocprofv3 kernel-trace + stats for one command, run from the repo root.
#   tools/prof_stats.sh <outname> <python args...>
# writes gpurun_out/prof/<outname>/... and prints a short per-kernel summary.
set -o pipefail
name=$1; shift
export TMPDIR=/tmp
out=gpurun_out/prof/$name
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python3 "$@" > $out/log.txt 2>&1 || { echo "rocprofv3 failed rc=$?"; tail -5 $out/log.txt; exit 1; }
f=$(find $out -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] || { echo "no kernel_stats.csv"; exit 1; }
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs'])/1e3:9.2f} min_us={float(r['MinNs'])/1e3:9.2f} pct={float(r['Percentage']):6.2f}")
PY
