"""Sum rocprofv3 counter_collection.csv rows per kernel and counter: tools/pmc_sum.py <dir> [label]"""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"].split("(")[0][:60], r["Counter_Name"])] += float(r["Counter_Value"])
label = sys.argv[2] if len(sys.argv) > 2 else ""
for (k, c), v in sorted(agg.items()):
    if "blind_rotate" in k or "ntt" in k:
        print(f"{label:10s} {k:60s} {c:24s} {v:.5g}")
