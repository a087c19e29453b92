"""Summarise rocprofv3 PMC passes (tools/pmc_run.sh) into profiles/<round>_pmc_traffic.json.

hbm_bytes_per_launch = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes).  The factor 2 is the gfx950
FETCH_SIZE correction (MI355X_MICROARCH.md, HBM section), re-measured here by build/calib_fetch:
streaming 512 MiB with 4-, 8- and 16-byte lanes reports 262,1xx KiB each; WRITE_SIZE reports the
bytes exactly.  FETCH_SIZE counts L2 -> fabric requests, so Infinity-Cache hits are included:
the figure is an upper bound on DRAM traffic.
valu_busy (pass p1) = SQ_ACTIVE_INST_VALU x 4 (the counter's quad-cycles) / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8
XCDs): the fraction of the kernel's cycles each SIMD spends issuing VALU instructions.
usage: python tools/pmc_traffic.py <round tag> <batch> [pmc dir]"""
import collections
import csv
import json
import os
import re
import sys

tag, batch = sys.argv[1], int(sys.argv[2])
d = sys.argv[3] if len(sys.argv) > 3 else "gpurun_out/pmc"
NTT_POLYS = 4096  # tools/pmc_workload.py


def per_kernel(pas, counter):
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, pas, "run_counter_collection.csv"))):
        if r["Counter_Name"] == counter:
            vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return vals


def short(name):
    """the names bench.py reports: k_blind_rotate_ginx, k_ntt1024w<fwd, SignedA>, k_ntt1024w64<inv>, ..."""
    m = re.search(r"(k_[a-z0-9_]+)", name)
    if not m:
        return name[:40]
    base = m.group(1)
    if base.startswith("k_ntt1024"):
        args = name[name.index(base) + len(base):].split("(")[0] + name.split(">(")[0]
        inv = "inv" if re.search(r"<\s*(unsigned long, )?true", name) else "fwd"
        if base == "k_ntt1024w64":
            return f"k_ntt1024w64<{inv}>"
        if base == "k_ntt1024w":
            arith = "SignedA" if "SignedA" in name else "ShoupA"
            return f"k_ntt1024w<{inv}, {arith}>"
        return f"k_ntt1024<{'uint64_t' if 'unsigned long,' in name else 'uint32_t'}, {inv}>"
    return base


fetch, write = per_kernel("p3", "FETCH_SIZE"), per_kernel("p4", "WRITE_SIZE")
cf, cw = per_kernel("c3", "FETCH_SIZE"), per_kernel("c4", "WRITE_SIZE")
calib = {short(k): {"fetch_kib": v[0]} for k, v in cf.items() if "k_read" in k}
for k, v in cw.items():
    if "k_write" in k:
        calib.setdefault(short(k), {})["write_kib"] = v[0]
out = {"round": tag, "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE --kernel-trace (separate passes)",
       "correction": "hbm_bytes = 2 * FETCH_SIZE_KiB * 1024 + WRITE_SIZE_KiB * 1024",
       "calibration_bytes": 512 << 20, "calibration": calib, "kernels": {}}
for k in fetch:
    if not k.startswith("fhe_amd::") and "fhe_amd::" not in k:
        continue
    f = sum(fetch[k]) / len(fetch[k])
    w = sum(write.get(k, [0])) / max(1, len(write.get(k, [0])))
    key = short(k)
    out["kernels"][key] = {
        "kernel": key, "batch": NTT_POLYS if "ntt" in key else batch, "launches": len(fetch[k]),
        "fetch_kib": round(f, 1), "write_kib": round(w, 1),
        "hbm_bytes_per_launch": round(2 * f * 1024 + w * 1024)}
valu, gui, insts = per_kernel("p1", "SQ_ACTIVE_INST_VALU"), per_kernel("p1", "GRBM_GUI_ACTIVE"), per_kernel("p1", "SQ_INSTS_VALU")
for k in valu:
    key = short(k)
    if key in out["kernels"] and gui.get(k):
        v, gcy = sum(valu[k]) / len(valu[k]), sum(gui[k]) / len(gui[k])
        out["kernels"][key]["valu_busy"] = round(v * 4 / 1024 / (gcy / 8), 4)
        out["kernels"][key]["valu_insts_per_launch"] = round(sum(insts[k]) / len(insts[k]))
path = os.path.join("profiles", f"{tag}_pmc_traffic.json")
json.dump(out, open(path, "w"), indent=1)
print(json.dumps(out["kernels"], indent=1))
