"""Per-kernel, per-grid-size summary of a rocprofv3 kernel trace (run_kernel_trace.csv): the
bench runs the blind-rotation kernel at two batch sizes (65,536 gates and config 3's 1,024), so
its --stats average mixes them; grouped by grid size each average matches one bench object.
usage: python tools/trace_by_grid.py <kernel_trace.csv> [out.csv]"""
import collections
import csv
import re
import sys

rows = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
    m = re.search(r"(k_[a-z0-9_]+)(<[^(]*?>)?\(", name)
    short = (m.group(1) + (m.group(2) or "")) if m else name[:60]
    grid = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
    rows[(short, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
out = [("kernel", "workgroups", "calls", "avg_us", "min_us", "max_us")]
for (k, g), v in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
    out.append((k, g, len(v), round(sum(v) / len(v), 2), round(min(v), 2), round(max(v), 2)))
w = csv.writer(open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout)
w.writerows(out)
