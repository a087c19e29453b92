#!/usr/bin/env python3
"""bench.py -- TFHE gate bootstraps/sec (STD128) on MI355X, driver contract.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--total T | --batch B]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

With --gpus N > 1 and no launcher (WORLD_SIZE unset) bench.py starts the torch.distributed.run
child itself (N ranks, one per GPU) and exits with its return code.

A step = one EvalBinGate(AND) pass over BASELINE config 4's global batch of T = 65,536
independent STD128 GINX gate pairs, sharded contiguously over the N ranks (strong
scaling: T / N gates per GPU, no data-path collective), inputs resident in HBM:
gate prep + blind rotation (k_blind_rotate_ginx), then key switch + ModSwitch
(k_keyswitch_tiled).  Rank 0 prints ONE JSON line.  In the same line:

  * roofline       -- the dominant kernel (blind rotation): algorithmic bytes / launch
                      time (HIP events on the launch stream) vs HBM peak; tiny by
                      construction (the BSK is reused by every gate of the batch);
  * valu_roofline  -- the same kernel against the bound that binds: modular multiplies/s
                      vs the half-rate 32-bit integer multiply issue peak;
  * lmkcdey        -- BASELINE config 5: the same step on STD128_LMKCDEY (T gates,
                      same sharding), with its own roofline / valu_roofline / cpu_baseline;
  * config3        -- BASELINE config 3: B = 1024 GINX gates on one GPU (N = 1 only; warmup at least 0.2 s);
  * small_batch    -- one gate's latency on the default (two- / four-waves-per-gate) kernels of STD128 GINX and
                      STD128_LMKCDEY and on the one-wave kernels (N = 1 only);
  * ntt_roofline   -- BASELINE config 2: 4096-polynomial N = 1024 NTT and iNTT passes,
                      27-bit STD128 modulus (k_ntt1024w) and 60-bit poly-benchmark prime
                      (k_ntt1024w64), GB/s vs HBM peak;
  * cpu_baseline   -- the reference's own CPU path (oracle/_ref/libfhe_ref.so, built
                      from /root/reference) on this host, rank 0, N = 1 only: all cores
                      available to the job and 1 core, host model recorded; config-1
                      single-NTT time.
  * bit_exact_vs_reference -- the whole step's outputs hashed against the reference's
                      outputs for the same 65,536 gates (tests/golden/full_*.npz).
"""
import argparse
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "TFHE gate bootstraps/sec (STD128) at 1/2/4/8 MI355X; NTT GB/s vs HBM peak"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
VALU_MODMUL_PEAK_T = 256 * 4 * 16 * 2.4e9 / 3 / 1e12  # 13.1 T modmul/s (half-rate 32-bit multiplies)
# algorithmic bytes (reference u64 accounting)
BSK_BYTES = {"ginx": 65_929_216, "lmkcdey": 29_655_040}
KSK_BYTES = {"ginx": 396_361_728, "lmkcdey": 352_321_536}
IN_BYTES_PER_GATE = {"ginx": 2 * 504 * 8, "lmkcdey": 2 * 448 * 8}  # two LWE inputs (n+1 u64)
OUT_BYTES_PER_GATE = {"ginx": 504 * 8, "lmkcdey": 448 * 8}
EXT_BYTES_PER_GATE = 1025 * 8                                       # ctExt (N+1 u64)
NTT_BYTES_PER_POLY = 2 * 1024 * 8                                   # read + write u64
MODMUL_PER_GATE = {"ginx": 25.8e6, "lmkcdey": 24.7e6}              # SURVEY.md 8(a) cost table
K1_NAME = {"ginx": "k_blind_rotate_ginx", "lmkcdey": "k_blind_rotate_lmk"}
PREP_NAME = {"ginx": "k_prep_ginx", "lmkcdey": "k_prep_lmk_w"}
FULL_SHARD = 8192


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--total", type=int, default=65536, help="global gates per step (strong scaling)")
    ap.add_argument("--batch", type=int, default=0, help="gates per GPU per step (weak scaling; overrides --total)")
    ap.add_argument("--method", default="ginx", choices=["ginx", "lmkcdey"], help="method of the main line")
    ap.add_argument("--no-lmkcdey", action="store_true", help="skip the config-5 sub-object")
    ap.add_argument("--no-config3", action="store_true")
    ap.add_argument("--ntt-count", type=int, default=4096)
    ap.add_argument("--cpu-sample", type=int, default=8192, help="gates in the all-cores CPU sample (BASELINE.md 2)")
    ap.add_argument("--cpu-sample-1core", type=int, default=24, help="gates in the 1-core CPU sample")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: every core available to this job")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-small-batch", action="store_true", help="skip the one-gate latency sub-object")
    return ap.parse_args()


# ---------------------------------------------------------------------------------------------
# inputs: the seeded batch of tests/golden/make_golden.py full_inputs(), so the outputs can be
# checked against the reference's hashes for the same 65,536 gates
# ---------------------------------------------------------------------------------------------
def make_inputs(bf, ps, method, total):
    key_seed = 0xB0070000 + ps
    keys = bf.keygen(ps, method, key_seed)
    rng = np.random.default_rng(0xF011 + ps)
    x1, x2 = rng.integers(0, 2, total), rng.integers(0, 2, total)
    a1, b1 = bf.encrypt(ps, method, keys.sk, x1, 0xF0110000 + ps)
    a2, b2 = bf.encrypt(ps, method, keys.sk, x2, 0xF0120000 + ps)
    return keys, x1, x2, a1, b1, a2, b2


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.uint64).tobytes()).hexdigest()


def golden_check(name, lo, hi, total, ao, bo):
    """True/False when [lo, hi) of the 65,536-gate batch is covered by the reference hashes of
    tests/golden/full_<name>.npz (whole batch or whole 8192-gate shards), else None."""
    f = os.path.join(ROOT, "tests", "golden", f"full_{name}.npz")
    if not os.path.exists(f):
        return None
    g = np.load(f)
    if total != int(g["count"]):
        return None
    if lo == 0 and hi == total:
        return _sha(ao) + _sha(bo) == str(g["out_sha"])
    S = int(g["shard"])
    if lo % S or (hi - lo) % S:
        return None
    shards = [str(s) for s in g["shard_sha"]]
    return all(_sha(ao[s - lo:s - lo + S]) + _sha(bo[s - lo:s - lo + S]) == shards[s // S] for s in range(lo, hi, S))


def run_config(args, bf, torch, ctx, method_name, total, lo, hi, golden=None, min_warm_s=0.0):
    """Times K steps of EvalBinGate(AND) over gates [lo, hi) of a `total`-gate batch on this
    rank; returns the per-rank measurements (elapsed is max-reduced by the caller).  golden: the
    tests/golden/full_<golden>.npz reference hashes the outputs are checked against (default: the
    65,536-gate batch of the method).  min_warm_s: the warmup also lasts at least this long (config 3's
    4 ms steps: after the seconds of host-side setup the GPU clocks ramp up over its first ~25 ms,
    tools/c3_ramp.py, profiles/r06_c3_ramp.txt)."""
    from fhe_amd.dist import barrier
    dev, stream, sp = ctx["dev"], ctx["stream"], ctx["stream"].cuda_stream
    ps, method = (bf.STD128, bf.GINX) if method_name == "ginx" else (bf.STD128_LMKCDEY, bf.LMKCDEY)
    P = bf.params(ps, method)
    B = hi - lo
    t0 = time.time()
    keys, x1, x2, a1, b1, a2, b2 = make_inputs(bf, ps, method, total)
    eng = bf.GateEngine(ps, method, device=dev.index)
    eng.load_keys(keys.bsk, keys.kskA, keys.kskB)
    to_dev = lambda x: torch.from_numpy(np.ascontiguousarray(x[lo:hi]).view(np.int64)).to(dev)  # noqa: E731
    d_in = [to_dev(x) for x in (a1, b1, a2, b2)]
    d_ao = torch.empty((B, P.n), dtype=torch.int64, device=dev)
    d_bo = torch.empty((B,), dtype=torch.int64, device=dev)
    ptrs = [t.data_ptr() for t in d_in]
    log(f"[{method_name}] setup {time.time() - t0:.1f}s (keygen + upload), gates [{lo}, {hi}) of {total}")

    def step(ev=None):
        if ev:
            ev[0].record(stream)
        eng.blind_rotate_device(bf.AND, B, *ptrs, stream=sp)
        if ev:
            ev[1].record(stream)
        eng.keyswitch_workspace_device(B, d_ao.data_ptr(), d_bo.data_ptr(), stream=sp)
        if ev:
            ev[2].record(stream)

    t_warm, n_warm = time.perf_counter(), 0
    while n_warm < args.warmup or time.perf_counter() - t_warm < min_warm_s:
        step()
        n_warm += 1
        if min_warm_s:
            torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    torch.cuda.synchronize(dev)
    barrier()
    elapsed = time.perf_counter() - t_start
    br_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    ks_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))
    ao = d_ao.cpu().numpy().view(np.uint64)
    bo = d_bo.cpu().numpy().view(np.uint64)
    dec = bf.decrypt(ps, method, keys.sk, ao, bo)
    verified = bool(np.array_equal(dec, (x1[lo:hi] & x2[lo:hi]).astype(np.int64)))
    exact = golden_check(golden or ("std128" if method_name == "ginx" else "lmkcdey"), lo, hi, total, ao, bo)
    kernel = eng.gate_kernel(B)   # the blind-rotation kernel this batch launched (fhe_hip_gate_kernel)
    eng.close()
    return {"elapsed": elapsed, "br_ms": br_ms, "ks_ms": ks_ms, "verified": verified, "exact": exact, "B": B,
            "warmup_steps": n_warm,
            "keys": keys, "inputs": (a1[lo:hi], b1[lo:hi], a2[lo:hi], b2[lo:hi]), "out": (ao, bo), "ps": ps,
            "method": method, "kernel": kernel}


def per_gpu_hbm(method_name, B, step_s):
    """per-GPU compulsory bytes of a step = BSK + KSK + B x I/O (two LWE
    inputs and the output, reference u64 accounting; 561,381,376 B for GINX and 470,056,960 B for LMKCDEY at
    8192 gates) over the step time, against the HBM peak"""
    b = BSK_BYTES[method_name] + KSK_BYTES[method_name] + B * (IN_BYTES_PER_GATE[method_name] +
                                                               OUT_BYTES_PER_GATE[method_name])
    return {"bytes_per_gpu": b, "GBs": round(b / step_s / 1e9, 2), "frac": round(b / step_s / 1e9 / HBM_PEAK_GBS, 6),
            "basis": "BASELINE.md 3 (configs 4/5): BSK + KSK + shard x (two LWE inputs + output) per GPU / step "
                     "time (slowest rank); low by construction, the keys are reused by every gate"}


def rooflines(method_name, B, br_ms, ks_ms, kernel=None):
    """roofline (HBM) and valu_roofline of the blind-rotation kernel at B gates per launch (kernel: the name
    the context reports for the launch, default K1's)."""
    alg_bytes = BSK_BYTES[method_name] + B * (IN_BYTES_PER_GATE[method_name] + EXT_BYTES_PER_GATE)
    achieved = alg_bytes / (br_ms * 1e-3) / 1e9
    mm_rate = MODMUL_PER_GATE[method_name] * B / (br_ms * 1e-3) / 1e12
    k1 = kernel or K1_NAME[method_name]
    roofline = {
        "kernel": k1, "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": pmc_traffic(k1, B),
        "launch_ms": round(br_ms, 4), "launch_note": f"HIP events around {PREP_NAME[method_name]} + {k1} "
                                                     "(the prep kernel is <1% of it); max over ranks",
        "keyswitch_ms": round(ks_ms, 4),
        "alg_bytes_per_launch": alg_bytes,
        "alg_bytes_basis": "BSK (reference u64 accounting) + B x (two LWE inputs + ctExt), SURVEY 8(d)",
        "traffic_note": "2*FETCH_SIZE+WRITE_SIZE per launch from the committed rocprofv3 PMC summary "
                        "(profiles/*pmc_traffic.json, gfx950 FETCH correction), scaled to this batch; FETCH "
                        "counts L2->fabric requests incl. Infinity-Cache hits",
        "valu_note": "integer-VALU bound: see valu_roofline",
    }
    valu = {
        "kernel": k1, "bound": "valu-int-mul", "achieved": round(mm_rate, 3),
        "peak": round(VALU_MODMUL_PEAK_T, 4), "unit": "T modmul/s", "frac": round(mm_rate / VALU_MODMUL_PEAK_T, 4),
        "valu_busy_pmc": pmc_valu_busy(k1),
        "valu_busy_basis": "fraction of the kernel's cycles each SIMD issues VALU instructions (rocprofv3 PMC "
                           "SQ_ACTIVE_INST_VALU x 4 / 1024 SIMDs over GRBM_GUI_ACTIVE / 8 XCDs, committed summary "
                           "profiles/*pmc_traffic.json): the kernel is issue-bound at its instruction mix when this "
                           "is near 1",
        "basis": "SURVEY 8(a) modular multiplies per gate x gates / launch time; peak = 256 CUs x 4 SIMDs x "
                 "16 lanes/clk (half-rate 32-bit multiplies) x 2.4 GHz / 3 multiplies per modmul; the measured "
                 "multiply issue rate (profiles/archive/r01_ubench_valu_rates.txt, 35.1 T lane-op/s) is 11.7 T modmul/s",
    }
    return roofline, valu


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(args):
    """`python bench.py --gpus N` (N > 1) without a launcher: run N ranks, one process per GPU, as a
    torch.distributed.run child (started before anything touches the GPU: device_count() does not
    initialise it), relay its output and exit with its return code.  Fewer than N devices is an
    error unless FHE_BENCH_DEVICE_MAP places the ranks (the one-GPU rehearsal)."""
    import subprocess
    import torch
    have = torch.cuda.device_count()
    dmap = os.environ.get("FHE_BENCH_DEVICE_MAP")
    if dmap:
        devs = [int(x) for x in dmap.split(",")]
        if len(devs) < args.gpus or max(devs) >= have:
            log(f"error: FHE_BENCH_DEVICE_MAP={dmap} does not place {args.gpus} ranks on the {have} device(s)")
            return 2
    elif have < args.gpus:
        log(f"error: --gpus {args.gpus} but only {have} GPU(s) are visible")
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    log("launching", args.gpus, "ranks:", " ".join(cmd))
    return subprocess.call(cmd, env=dict(os.environ))


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    import torch
    import torch.distributed as dist

    from fhe_amd.dist import max_over_ranks, shard
    rank, world, local = env_rank()
    if world != args.gpus:
        log(f"error: WORLD_SIZE={world} differs from --gpus={args.gpus}")
        sys.exit(2)
    # rehearsal knobs (not used by the driver): FHE_BENCH_DEVICE_MAP="0,0" puts ranks on
    # chosen devices, FHE_BENCH_BACKEND=gloo for a one-GPU box
    dmap = os.environ.get("FHE_BENCH_DEVICE_MAP")
    env_local = local
    if dmap:
        local = int(dmap.split(",")[local])
    backend = os.environ.get("FHE_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    red_dev = dev if backend == "nccl" else None
    # which devices the ranks ran on, as the process group saw them (the driver's N-GPU line must show N
    # distinct GPUs under RCCL; a rank sharing a device with another is refused there, marked a rehearsal here)
    from fhe_amd.dist import check_topology, device_identity, gather_identities, topology_record
    topo = topology_record(gather_identities(device_identity(torch, dev, rank, env_local)),
                           backend if world > 1 else None, rehearsal=bool(dmap))
    try:
        check_topology(topo)
    except RuntimeError as e:
        log(f"error: {e}")
        sys.exit(3)
    stream = torch.cuda.Stream(dev)     # a real (non-null) stream: our kernels launch on it and
    assert stream.cuda_stream, "need a non-default stream handle"   # the timing events are recorded on it
    ctx = {"dev": dev, "stream": stream}

    from fhe_amd import binfhe as bf
    from fhe_amd import NttPlan

    if args.batch:
        total, scaling = args.batch * world, "weak"
    else:
        total, scaling = args.total, "strong"
    lo, hi = shard(total, rank, world)

    def measure(method_name):
        r = run_config(args, bf, torch, ctx, method_name, total, lo, hi)
        # launch times as well: the roofline of an N-rank line is the slowest rank's kernel
        el, bad, inexact, unknown, br, ks = max_over_ranks(
            [r["elapsed"], 0.0 if r["verified"] else 1.0, 1.0 if r["exact"] is False else 0.0,
             1.0 if r["exact"] is None else 0.0, r["br_ms"], r["ks_ms"]], device=red_dev)
        r["elapsed"], r["br_ms"], r["ks_ms"] = el, br, ks
        r["verified"] = bad == 0.0
        r["exact"] = None if unknown else inexact == 0.0
        return r

    main_r = measure(args.method)
    lmk_r = measure("lmkcdey") if (args.method == "ginx" and not args.no_lmkcdey) else None

    result = None
    if rank == 0:
        roofline, valu = rooflines(args.method, main_r["B"], main_r["br_ms"], main_r["ks_ms"], main_r["kernel"])
        value = total * args.steps / main_r["elapsed"]
        result = {
            "metric": METRIC, "value": round(value, 1), "unit": "bootstraps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(main_r["elapsed"] / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "u32",
            "data": "synthetic: seeded keys (fhe_amd keygen) and seeded random-bit encryptions, the batch of "
                    "tests/golden/full_*.npz",
            "config": {"workload": f"STD128{'' if args.method == 'ginx' else '_LMKCDEY'} {args.method.upper()} "
                                   f"EvalBinGate(AND), {total} gates per step over {world} GPU(s) "
                                   f"({hi - lo} per GPU; BASELINE config {'4' if args.method == 'ginx' else '5'})",
                       "paramset": "STD128" if args.method == "ginx" else "STD128_LMKCDEY",
                       "method": args.method.upper(), "global_batch": total, "batch_per_gpu": hi - lo,
                       "parallelism": f"shard{world}"},
            "verified": main_r["verified"],
            "bit_exact_vs_reference": main_r["exact"],
            "roofline": roofline,
            "valu_roofline": valu,
            "hbm_per_gpu": per_gpu_hbm(args.method, hi - lo, main_r["elapsed"] / args.steps),
            "distributed": topo,
        }
        if lmk_r is not None:
            lr, lv = rooflines("lmkcdey", lmk_r["B"], lmk_r["br_ms"], lmk_r["ks_ms"], lmk_r["kernel"])
            result["lmkcdey"] = {
                "config": f"BASELINE config 5: STD128_LMKCDEY EvalBinGate(AND), {total} gates per step over "
                          f"{world} GPU(s) ({hi - lo} per GPU)",
                "value": round(total * args.steps / lmk_r["elapsed"], 1), "unit": "bootstraps/s",
                "ms_per_step": round(lmk_r["elapsed"] / args.steps * 1e3, 3),
                "verified": lmk_r["verified"], "bit_exact_vs_reference": lmk_r["exact"],
                "roofline": lr, "valu_roofline": lv, "cpu_baseline": None,
                "hbm_per_gpu": per_gpu_hbm("lmkcdey", hi - lo, lmk_r["elapsed"] / args.steps),
            }
    if world == 1 and not args.no_config3 and args.method == "ginx":
        c3 = run_config(args, bf, torch, ctx, "ginx", 1024, 0, 1024, golden="std128_b1024", min_warm_s=0.2)
        r3, v3 = rooflines("ginx", 1024, c3["br_ms"], c3["ks_ms"], c3["kernel"])
        alg3 = BSK_BYTES["ginx"] + KSK_BYTES["ginx"] + 1024 * (IN_BYTES_PER_GATE["ginx"] + OUT_BYTES_PER_GATE["ginx"])
        step_s = c3["elapsed"] / args.steps
        result["config3"] = {
            "config": "BASELINE config 3: STD128 GINX EvalBinGate(AND), 1024 gates, 1 GPU",
            "value": round(1024 / step_s, 1), "unit": "bootstraps/s", "ms_per_step": round(step_s * 1e3, 3),
            "warmup_steps": c3["warmup_steps"], "warmup_rule": "max(W steps, 0.2 s): steady clocks (profiles/r06_c3_ramp.txt)",
            "verified": c3["verified"], "bit_exact_vs_reference": c3["exact"],
            "valu_roofline": v3, "blind_rotate_ms": r3["launch_ms"],
            "keyswitch_ms": r3["keyswitch_ms"],
            "hbm_frac_compulsory": round(alg3 / step_s / 1e9 / HBM_PEAK_GBS, 6),
            "hbm_basis": "SURVEY 8(d) config 3: BSK + KSK + 1024 x I/O = 474,677,248 B per batch / step time",
        }
    if rank == 0 and world == 1:
        if not args.no_small_batch:
            result["small_batch"] = small_batch(bf, torch, dev, stream)
        result["ntt_roofline"] = ntt_rooflines(NttPlan, torch, dev, stream, args.ntt_count)
        result["copy_bw"] = copy_bandwidth(torch, dev, stream, args.ntt_count)
        cpu = None
        if not args.no_cpu_baseline:
            cpu = cpu_baseline(main_r, args)
            if lmk_r is not None:
                result["lmkcdey"]["cpu_baseline"] = cpu_baseline(lmk_r, args)
        result["cpu_baseline"] = cpu
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        from fhe_amd.dist import barrier
        barrier()
        dist.destroy_process_group()
    return result


def env_rank():
    from fhe_amd.dist import env
    return env()


def pmc_summary(kernel, field):
    """`field` of `kernel` in the newest committed rocprofv3 PMC summary that has it
    (profiles/*pmc_traffic.json, written by tools/pmc_traffic.py; r03 after r02), with that
    summary's batch; (None, None) if not measured."""
    import glob
    best = (None, None)
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic*.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        # tools/pmc_traffic.py writes {"round", "calibration", ..., "kernels": {name: {...}}}; a summary committed
        # as that tool's stdout is the bare {name: {...}} map
        ks = d.get("kernels") if isinstance(d.get("kernels"), dict) else d
        k = ks.get(kernel) if isinstance(ks, dict) else None
        if isinstance(k, dict) and k.get("batch") and k.get(field) is not None:
            best = (k[field], k["batch"])
    return best


def pmc_traffic(kernel, batch):
    """HBM bytes per launch from the committed PMC summary, scaled to this batch; None if not measured"""
    v, b = pmc_summary(kernel, "hbm_bytes_per_launch")
    return None if v is None else round(v / b * batch)


def pmc_valu_busy(kernel):
    """the kernel's VALU issue fraction from the committed PMC summary (SQ_ACTIVE_INST_VALU x 4 per SIMD
    over GRBM_GUI_ACTIVE per XCD, tools/pmc_traffic.py); None if not measured"""
    return pmc_summary(kernel, "valu_busy")[0]


def small_batch(bf, torch, dev, stream, reps=20):
    """Latency of one gate (EvalBinGate(AND): prep, blind rotation, key switch; inputs resident, HIP events on
    the stream, median of `reps`) on the default kernels of STD128 GINX and STD128_LMKCDEY (the two- and
    four-waves-per-gate forms) and on the one-wave kernels they replace below two
    gates per CU (FHE_HIP_{GINX,LMK}_KERNEL=wave); checked by decryption."""
    out = {"gates": 1, "unit": "ms", "basis": "median of %d single-gate calls, HIP events on the stream" % reps}
    sp = stream.cuda_stream
    for name, ps, m, knob in (("ginx", bf.STD128, bf.GINX, "FHE_HIP_GINX_KERNEL"),
                              ("lmkcdey", bf.STD128_LMKCDEY, bf.LMKCDEY, "FHE_HIP_LMK_KERNEL")):
        keys = bf.keygen(ps, m, 0x5B00 + ps)
        P = bf.params(ps, m)
        a1, b1 = bf.encrypt(ps, m, keys.sk, np.array([1]), 11)
        a2, b2 = bf.encrypt(ps, m, keys.sk, np.array([1]), 12)
        d_in = [torch.from_numpy(np.ascontiguousarray(x).view(np.int64)).to(dev) for x in (a1, b1, a2, b2)]
        d_ao = torch.empty((1, P.n), dtype=torch.int64, device=dev)
        d_bo = torch.empty((1,), dtype=torch.int64, device=dev)
        for kind in ("default", "wave"):
            if kind == "wave":
                os.environ[knob] = "wave"
            try:
                eng = bf.GateEngine(ps, m, device=dev.index)
            finally:
                os.environ.pop(knob, None)
            eng.load_keys(keys.bsk, keys.kskA, keys.kskB)
            ts = []
            for k in range(reps + 40):  # 40 warmup calls: steady clocks (profiles/r06_c3_ramp.txt)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                eng.eval_gate_device(bf.AND, 1, *[t.data_ptr() for t in d_in], d_ao.data_ptr(), d_bo.data_ptr(),
                                     stream=sp)
                e1.record(stream)
                e1.synchronize()
                if k >= 40:
                    ts.append(e0.elapsed_time(e1))
            ao = d_ao.cpu().numpy().view(np.uint64)
            bo = d_bo.cpu().numpy().view(np.uint64)
            ok = bool(bf.decrypt(ps, m, keys.sk, ao, bo)[0] == 1)
            out[f"{name}_{kind}"] = {"ms": round(float(np.median(ts)), 3), "kernel": eng.gate_kernel(1), "verified": ok}
            eng.close()
    return out


def ntt_rooflines(NttPlan, torch, dev, stream, count, reps=20):
    """BASELINE config 2: forward and inverse passes over `count` polynomials for the STD128 modulus
    (27-bit, k_ntt1024w SignedA) and the poly-benchmark 60-bit prime (k_ntt1024w64)."""
    out = []
    sp = stream.cuda_stream
    for Q, kname in ((134215681, "k_ntt1024w<{}, SignedA>"), (1152921504606830593, "k_ntt1024w64<{}>")):
        plan = NttPlan(Q, device=dev.index)
        x = torch.randint(0, min(Q, 2**62), (count, 1024), dtype=torch.int64, device=dev)
        for inv in (False, True):   # in place, as SwitchFormat transforms a polynomial in place
            for _ in range(3):
                plan.run_device(x.data_ptr(), x.data_ptr(), count, inv, stream=sp)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                plan.run_device(x.data_ptr(), x.data_ptr(), count, inv, stream=sp)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            ms = e0.elapsed_time(e1) / reps
            ach = count * NTT_BYTES_PER_POLY / (ms * 1e-3) / 1e9
            name = kname.format("inv" if inv else "fwd")
            out.append({"kernel": name, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                        "traffic": pmc_traffic(name, count), "valu_busy_pmc": pmc_valu_busy(name),
                        "launch_us": round(ms * 1e3, 3), "polys": count,
                        "Q": Q, "alg_bytes_per_launch": count * NTT_BYTES_PER_POLY})
        plan.close()
    return out


def copy_bandwidth(torch, dev, stream, count, reps=50):
    """measured device copy bandwidth (record it next to the 8 TB/s vendor peak): torch's
    copy of the bytes of one 4096-polynomial NTT pass (32 MiB read + 32 MiB written), on the bench stream"""
    x = torch.empty(count * 1024, dtype=torch.int64, device=dev)
    y = torch.empty_like(x)
    with torch.cuda.stream(stream):
        for _ in range(5):
            y.copy_(x)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            y.copy_(x)
        e1.record(stream)
    torch.cuda.synchronize(dev)
    us = e0.elapsed_time(e1) / reps * 1e3
    gbs = 2 * x.numel() * 8 / (us * 1e-6) / 1e9
    return {"bytes_per_copy": 2 * x.numel() * 8, "us": round(us, 3), "GBs": round(gbs, 1),
            "frac_of_peak": round(gbs / HBM_PEAK_GBS, 4), "method": "torch copy_ on the bench stream, 50 reps"}


def host_info():
    """CPU facts of this host: the whole machine and what this job may use."""
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except Exception:
        info["affinity"] = None
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(p)
    except Exception:
        pass
    info["cgroup_cpus"] = quota
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                info["model"] = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    avail = info["affinity"] or info["nproc"] or 1
    if quota:
        avail = max(1, min(avail, int(quota)))
    info["usable"] = avail
    return info


def cpu_baseline(r, args):
    """The reference's CPU path on this host: EvalBinGateBatch semantics (OpenMP parallel-for over
    BinFHEContext::EvalBinGate, batch.cpp:197-200) on bounded samples of the same batch, on every
    core available to the job and on 1 core; plus the config-1 single-NTT time."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import Ref, Restatement, ref_available, restatement_available
    hi = host_info()
    threads = args.cpu_threads or hi["usable"]
    ps, method, keys = r["ps"], r["method"], r["keys"]
    a1, b1, a2, b2 = r["inputs"]
    ao, bo = r["out"]
    label = "GINX" if method == 2 else "LMKCDEY"
    S_all = min(args.cpu_sample, len(b1))
    S_one = min(args.cpu_sample_1core if method == 2 else max(1, args.cpu_sample_1core * 2 // 3), len(b1))
    if ref_available():
        ref = Ref(ps, method)
        ref.load_keys(keys.bsk, keys.kskA, keys.kskB)
        ref.time_gates(1, a1[:2], b1[:2], a2[:2], b2[:2], nthreads=min(2, threads))   # warm-up (tables)
        t_all, ra, rb = ref.time_gates(1, a1[:S_all], b1[:S_all], a2[:S_all], b2[:S_all], nthreads=threads)
        off = S_all
        S_one = min(S_one, len(b1) - off) if len(b1) > off else S_one
        sl1 = slice(off, off + S_one) if len(b1) > off else slice(0, S_one)
        t_one, ra1, rb1 = ref.time_gates(1, a1[sl1], b1[sl1], a2[sl1], b2[sl1], nthreads=1)
        kind = "reference"
    elif restatement_available():
        O = Restatement(ps, method)
        t0 = time.perf_counter()
        ra, rb = O.eval_gate(keys.bsk, keys.kskA, keys.kskB, 1, a1[:S_all], b1[:S_all], a2[:S_all], b2[:S_all],
                             nthreads=threads)
        t_all = time.perf_counter() - t0
        sl1 = slice(0, S_one)
        t0 = time.perf_counter()
        ra1, rb1 = O.eval_gate(keys.bsk, keys.kskA, keys.kskB, 1, a1[sl1], b1[sl1], a2[sl1], b2[sl1], nthreads=1)
        t_one = time.perf_counter() - t0
        ref = None
        kind = "port"
    else:
        return None
    match = bool(np.array_equal(ra, ao[:S_all]) and np.array_equal(rb, bo[:S_all])
                 and np.array_equal(ra1, ao[sl1]) and np.array_equal(rb1, bo[sl1]))
    out = {"value": round(S_all / t_all, 2), "unit": "bootstraps/s", "cores": threads, "kind": kind,
           "sample": f"{S_all} STD128{'' if method == 2 else '_LMKCDEY'} {label} AND gates of the same batch, "
                     f"OpenMP parallel-for over EvalBinGate on {threads} threads ({t_all:.2f} s wall); 1-core leg: "
                     f"{S_one} gates ({t_one:.2f} s)",
           "value_1core": round(S_one / t_one, 3), "ms_per_gate_1core": round(t_one / S_one * 1e3, 2),
           "host": hi, "bit_exact_vs_gpu": match}
    if method == 2 and ref is not None:
        # config 1 (poly-benchmark Native_ntt body, poly-benchmark.h:213-221): one N = 1024 forward
        # NTT on one core, 60-bit and STD128 moduli; config 2 CPU cost = 4096 x that
        ntt = {}
        rng = np.random.default_rng(0x5EED0001)
        ref.L.ref_ntt_batch_bench.restype = ctypes.c_double
        ref.L.ref_ntt_batch_bench.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t,
                                              ctypes.c_int]
        for nm, Q in (("q60", 1152921504606830593), ("std128", 134215681)):
            x = rng.integers(0, Q, size=1024, dtype=np.uint64)
            ns = ref.L.ref_ntt_bench(Q, 1024, x.ctypes.data, 20000)
            xb = rng.integers(0, Q, size=(4096, 1024), dtype=np.uint64)
            ref.L.ref_ntt_batch_bench(Q, 1024, xb.ctypes.data, 4096, threads)   # warm-up
            nsb = min(ref.L.ref_ntt_batch_bench(Q, 1024, xb.ctypes.data, 4096, threads) for _ in range(3))
            ntt[nm] = {"Q": Q, "us_per_ntt_1core": round(ns / 1e3, 3),
                       "config2_us_4096_1core": round(ns * 4096 / 1e3, 1),
                       "config2_us_4096_all_cores": round(nsb / 1e3, 1), "all_cores_threads": threads,
                       "config2_GBs_all_cores": round(4096 * NTT_BYTES_PER_POLY / (nsb * 1e-9) / 1e9, 2)}
        out["ntt_config1"] = ntt
    return out


if __name__ == "__main__":
    main()
