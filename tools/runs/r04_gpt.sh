#!/bin/bash
# Round 4: key switch with 2 / 4 gates per thread (1024- / 2048-gate tiles: KSK traffic / 2, / 4) vs the
# 512-gate tiles: time and output hash (tools/ks_time.py, interleaved), then FETCH/WRITE per launch
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04_gpt_ab.txt; : > $o
for r in 1 2; do
  for v in base gpt2 gpt4; do
    lib=""; [ $v != base ] && lib="FHE_AMD_LIB=abv/$v.so"
    echo -n "$v r$r: " >> $o; env $lib timeout -k 10 120 python -u tools/ks_time.py 65536 20 >> $o 2>&1 || exit 1
  done
done
cat $o
mkdir -p gpurun_out/pmc_gpt
for v in base gpt2 gpt4; do
  lib=""; [ $v != base ] && lib="abv/$v.so"
  for c in FETCH_SIZE WRITE_SIZE; do
    FHE_AMD_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_gpt/${v}_$c -o run -- python3 tools/ks_time.py 65536 2 > /dev/null 2>&1 || { echo "pmc $v $c failed"; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, collections
for v in ("base", "gpt2", "gpt4"):
    out = []
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        vals = collections.defaultdict(list)
        for f in glob.glob(f"gpurun_out/pmc_gpt/{v}_{c}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "keyswitch" in r["Kernel_Name"] and r["Counter_Name"] == c:
                    vals[r["Dispatch_Id"]].append(float(r["Counter_Value"]))
        per = [sum(x) for x in vals.values()]
        out.append((c, len(per), sum(per) / max(1, len(per))))
    fetch, write = out[0][2], out[1][2]
    print(f"{v}: launches={out[0][1]} FETCH_KiB={fetch:.0f} WRITE_KiB={write:.0f} traffic_GB={(2*fetch+write)*1024/1e9:.2f}")
PY
