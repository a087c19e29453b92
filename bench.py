#!/usr/bin/env python3
"""bench.py -- TFHE gate bootstraps/sec (STD128) on MI355X, driver contract.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--method ginx|lmkcdey]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

A step = one EvalBinGate(AND) pass over a batch of B independent gate pairs per
GPU (default B = 8192 = BASELINE.json config 4's per-GPU shard of 65536), inputs
resident in HBM: blind rotation (k_blind_rotate_*) then key switch
(k_keyswitch).  Ranks shard gates with no data-path collective ("weak"
scaling: B per GPU fixed).  Rank 0 prints one JSON line.

Also measured in the same run and reported beside `value`:
  * roofline     -- dominant kernel of the step (blind rotation): algorithmic
                    bytes / launch time (HIP events on the launch stream) vs HBM
                    peak (tiny by construction: the BSK is reused by every gate);
  * valu_roofline -- the same kernel against the bound that binds: modular
                    multiplies per second vs the 32-bit integer multiply issue peak;
  * ntt_roofline -- BASELINE config 2: batched N=1024 NTT x 4096, GB/s vs HBM peak;
  * cpu_baseline -- the reference's own CPU path (oracle/_ref/libfhe_ref.so,
                    built from /root/reference) on the host cores, rank 0, N=1.
"""
import argparse
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
KEY_SEED = 0xBE4C0001
# algorithmic bytes (reference u64 accounting)
BSK_BYTES = {"ginx": 65_929_216, "lmkcdey": 29_655_040}
IN_BYTES_PER_GATE = {"ginx": 2 * 504 * 8, "lmkcdey": 2 * 448 * 8}  # two LWE inputs (n+1 u64)
EXT_BYTES_PER_GATE = 1025 * 8                                       # ctExt (N+1 u64)
NTT_BYTES_PER_POLY = 2 * 1024 * 8                                   # read + write u64


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=8192, help="gates per GPU per step")
    ap.add_argument("--method", default="ginx", choices=["ginx", "lmkcdey"])
    ap.add_argument("--ntt-count", type=int, default=4096)
    ap.add_argument("--cpu-sample", type=int, default=3072, help="gates in the CPU-baseline sample (~12 s of host work)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from fhe_amd.dist import barrier, env, max_over_ranks
    rank, world, local = env()
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} differs from --gpus={args.gpus}; using WORLD_SIZE")
    # rehearsal knobs (not used by the driver): FHE_BENCH_DEVICE_MAP="0,0" puts ranks on
    # chosen devices, FHE_BENCH_BACKEND=gloo for a one-GPU box
    dmap = os.environ.get("FHE_BENCH_DEVICE_MAP")
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

    from fhe_amd import binfhe as bf
    from fhe_amd import NttPlan

    ps, method = (bf.STD128, bf.GINX) if args.method == "ginx" else (bf.STD128_LMKCDEY, bf.LMKCDEY)
    P = bf.params(ps, method)
    B = args.batch

    # ---- setup (untimed): keys replicated on every GPU, inputs resident in HBM
    t0 = time.time()
    keys = bf.keygen(ps, method, KEY_SEED)
    eng = bf.GateEngine(ps, method, device=local)
    eng.load_keys(keys.bsk, keys.kskA, keys.kskB)
    rng = np.random.default_rng(1000 + rank)
    x1, x2 = rng.integers(0, 2, B), rng.integers(0, 2, B)
    a1, b1 = bf.encrypt(ps, method, keys.sk, x1, 2000 + rank)
    a2, b2 = bf.encrypt(ps, method, keys.sk, x2, 3000 + rank)
    to_dev = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.int64)).to(dev)  # noqa: E731
    d_in = [to_dev(x) for x in (a1, b1, a2, b2)]
    d_ao = torch.empty((B, P.n), dtype=torch.int64, device=dev)
    d_bo = torch.empty((B,), dtype=torch.int64, device=dev)
    ptrs = [t.data_ptr() for t in d_in]
    stream = torch.cuda.Stream(dev)      # a real (non-null) stream: our kernels launch on it and
    sp = stream.cuda_stream              # the timing events are recorded on it
    assert sp, "need a non-default stream handle"
    log(f"[rank {rank}] setup {time.time() - t0:.1f}s (keygen + upload), batch {B}")

    def step(ev=None):
        if ev:
            ev[0].record(stream)
        eng.blind_rotate_device(bf.AND, B, *ptrs, stream=sp)
        if ev:
            ev[1].record(stream)
        eng.keyswitch_workspace_device(B, d_ao.data_ptr(), d_bo.data_ptr(), stream=sp)
        if ev:
            ev[2].record(stream)

    for _ in range(args.warmup):
        step()
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

    # correctness of the last step (host decrypt of the whole shard)
    ao = d_ao.cpu().numpy().view(np.uint64)
    bo = d_bo.cpu().numpy().view(np.uint64)
    verified = bool(np.array_equal(bf.decrypt(ps, method, keys.sk, ao, bo), (x1 & x2).astype(np.int64)))

    elapsed, bad = max_over_ranks([elapsed, 0.0 if verified else 1.0], device=red_dev)
    verified = bad == 0.0

    total_gates = B * world * args.steps
    value = total_gates / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    result = None
    if rank == 0:
        # ---- roofline of the dominant kernel (blind rotation), live HIP-event timing
        alg_bytes = BSK_BYTES[args.method] + B * (IN_BYTES_PER_GATE[args.method] + EXT_BYTES_PER_GATE)
        achieved = alg_bytes / (br_ms * 1e-3) / 1e9
        # integer-VALU view: modular multiplies per gate (SURVEY.md 8(a) cost table)
        mm_per_gate = 25.8e6 if args.method == "ginx" else 24.7e6
        roofline = {
            "kernel": f"k_blind_rotate_{args.method}",
            "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": pmc_traffic(f"k_blind_rotate_{args.method}", B),
            "launch_ms": round(br_ms, 4), "keyswitch_ms": round(ks_ms, 4),
            "alg_bytes_per_launch": alg_bytes,
            "traffic_note": "2*FETCH_SIZE+WRITE_SIZE (profiles/*pmc_traffic.json); FETCH counts L2->fabric "
                            "requests incl. Infinity-Cache hits: the BSK is streamed once per XCD per wave "
                            "generation (8 XCDs x 4 generations at B=8192) from the 256 MiB cache",
            "valu_note": "integer-VALU bound: see valu_roofline",
            "modmul_per_s": round(mm_per_gate * B / (br_ms * 1e-3) / 1e12, 3), "modmul_unit": "T/s",
        }
        # the bound that binds: 32-bit integer multiply issue (each modular multiply is three
        # half-rate multiplies: v_mad_i64_i32, v_mul_lo_u32, v_mad_i64_i32)
        mm_rate = mm_per_gate * B / (br_ms * 1e-3) / 1e12
        valu_roofline = {
            "kernel": f"k_blind_rotate_{args.method}", "bound": "valu-int-mul", "achieved": round(mm_rate, 3),
            "peak": VALU_MODMUL_PEAK_T, "unit": "T modmul/s", "frac": round(mm_rate / VALU_MODMUL_PEAK_T, 4),
            "basis": "SURVEY 8(a) modular multiplies per gate x gates / launch time; peak = 256 CUs x 4 SIMDs x "
                     "16 lanes/clk (half-rate 32-bit multiplies) x 2.4 GHz / 3 multiplies per modmul; the measured "
                     "multiply issue rate (profiles/r01_ubench_valu_rates.txt, 35.1 T lane-op/s) is 11.7 T modmul/s",
        }
        ntt = ntt_roofline(NttPlan, torch, dev, stream, args.ntt_count) if world == 1 else None
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(ps, method, keys, a1, b1, a2, b2, ao, bo, args)
        result = {
            "metric": METRIC, "value": round(value, 1), "unit": "bootstraps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic: seeded keys (fhe_amd keygen), random bit encryptions",
            "config": {"workload": f"STD128{'' if args.method == 'ginx' else '_LMKCDEY'} "
                                   f"{args.method.upper()} EvalBinGate(AND), {B} gates per GPU per step "
                                   f"(BASELINE config {'4' if args.method == 'ginx' else '5'} shard)",
                       "paramset": "STD128" if args.method == "ginx" else "STD128_LMKCDEY",
                       "method": args.method.upper(), "batch_per_gpu": B, "global_batch": B * world,
                       "parallelism": f"shard{world}"},
            "verified": verified,
            "roofline": roofline,
            "valu_roofline": valu_roofline,
            "ntt_roofline": ntt,
            "cpu_baseline": cpu,
        }
        print(json.dumps(result), flush=True)
    if world > 1:
        barrier()
        dist.destroy_process_group()
    return result


def pmc_traffic(kernel, batch):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/*pmc*.json,
    written by tools/pmc_traffic.py), scaled to this batch; None if not measured."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        k = d.get("kernels", {}).get(kernel)
        if k and k.get("batch"):
            best = k["hbm_bytes_per_launch"] / k["batch"] * batch
    return None if best is None else round(best)


def ntt_roofline(NttPlan, torch, dev, stream, count, reps=20):
    Q = 134215681
    plan = NttPlan(Q, device=dev.index)
    x = torch.randint(0, Q, (count, 1024), dtype=torch.int64, device=dev)
    sp = stream.cuda_stream
    for _ in range(3):
        plan.run_device(x.data_ptr(), x.data_ptr(), count, False, stream=sp)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        plan.run_device(x.data_ptr(), x.data_ptr(), count, False, stream=sp)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    ach = count * NTT_BYTES_PER_POLY / (ms * 1e-3) / 1e9
    plan.close()
    return {"kernel": "k_ntt1024w<fwd, SignedA>", "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": pmc_traffic("k_ntt1024w", count),
            "launch_us": round(ms * 1e3, 3), "polys": count, "Q": Q}


def cpu_baseline(ps, method, keys, a1, b1, a2, b2, ao, bo, args):
    """The reference's CPU path timed on this host: EvalBinGateBatch semantics (OpenMP
    parallel-for over BinFHEContext::EvalBinGate, batch.cpp:197-200) on a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import Ref, Restatement, ref_available, restatement_available
    S = min(args.cpu_sample, len(b1))
    threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    sl = slice(0, S)
    if ref_available():
        ref = Ref(ps, method)
        ref.load_keys(keys.bsk, keys.kskA, keys.kskB)
        t, ra, rb = ref.time_gates(1, a1[sl], b1[sl], a2[sl], b2[sl], nthreads=threads)
        kind = "reference"
    elif restatement_available():
        O = Restatement(ps, method)
        t0 = time.perf_counter()
        ra, rb = O.eval_gate(keys.bsk, keys.kskA, keys.kskB, 1, a1[sl], b1[sl], a2[sl], b2[sl], nthreads=threads)
        t = time.perf_counter() - t0
        kind = "port"
    else:
        return None
    match = bool(np.array_equal(ra, ao[sl]) and np.array_equal(rb, bo[sl]))
    return {"value": round(S / t, 2), "unit": "bootstraps/s", "cores": threads, "kind": kind,
            "sample": f"{S} STD128 {'GINX' if method == 2 else 'LMKCDEY'} AND gates of the same batch, "
                      f"OpenMP parallel-for over EvalBinGate, {threads} threads, {t:.2f} s wall",
            "bit_exact_vs_gpu": match}


if __name__ == "__main__":
    main()
