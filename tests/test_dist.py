"""Sharded (N>1) path on CPU with gloo, world_size 2: contiguous shards evaluated
per rank (by the oracle restatement, standing in for the GPU) reassemble to the
full-batch result; MAX-over-ranks timing reduction."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from fhe_amd.dist import shard


def test_shard_partition():
    for total in (0, 1, 7, 8192, 65536, 65537):
        for world in (1, 2, 3, 8):
            spans = [shard(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fhe_amd import binfhe as bf
    from fhe_amd.dist import barrier, max_over_ranks
    from oracle_lib import Restatement
    ps, m = bf.STD128, bf.GINX
    keys = bf.keygen(ps, m, 77)                    # replicated keys (same seed on every rank)
    total = 6
    rng = np.random.default_rng(9)                 # same global batch on every rank
    x1, x2 = rng.integers(0, 2, total), rng.integers(0, 2, total)
    a1, b1 = bf.encrypt(ps, m, keys.sk, x1, 1)
    a2, b2 = bf.encrypt(ps, m, keys.sk, x2, 2)
    lo, hi = shard(total, rank, world)
    O = Restatement(ps, m)
    barrier()
    ao, bo = O.eval_gate(keys.bsk, keys.kskA, keys.kskB, 1, a1[lo:hi], b1[lo:hi], a2[lo:hi], b2[lo:hi], nthreads=2)
    t = max_over_ranks([float(rank + 1)])
    barrier()
    np.savez(os.path.join(outdir, f"r{rank}.npz"), ao=ao, bo=bo, lo=lo, hi=hi, t=t[0])
    dist.destroy_process_group()


@pytest.mark.slow
def test_gloo_world2_sharded_gates(tmp_path, restatement):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    parts = [np.load(tmp_path / f"r{r}.npz") for r in range(world)]
    assert all(float(p["t"]) == float(world) for p in parts)       # MAX over ranks
    ao = np.concatenate([p["ao"] for p in parts])
    bo = np.concatenate([p["bo"] for p in parts])
    from fhe_amd import binfhe as bf
    from oracle_lib import Restatement
    keys = bf.keygen(bf.STD128, bf.GINX, 77)
    rng = np.random.default_rng(9)
    x1, x2 = rng.integers(0, 2, 6), rng.integers(0, 2, 6)
    a1, b1 = bf.encrypt(bf.STD128, bf.GINX, keys.sk, x1, 1)
    a2, b2 = bf.encrypt(bf.STD128, bf.GINX, keys.sk, x2, 2)
    fa, fb = Restatement(bf.STD128, bf.GINX).eval_gate(keys.bsk, keys.kskA, keys.kskB, 1, a1, b1, a2, b2)
    assert np.array_equal(ao, fa) and np.array_equal(bo, fb)
    assert np.array_equal(bf.decrypt(bf.STD128, bf.GINX, keys.sk, ao, bo), (x1 & x2).astype(np.int64))


def test_bench_refuses_more_ranks_than_devices():
    """`bench.py --gpus N` without a launcher starts N ranks itself; with fewer than N devices visible
    (none here) it fails loudly instead of measuring one rank"""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                            "FHE_BENCH_DEVICE_MAP")}
    import torch
    n = torch.cuda.device_count()      # counts without initialising the GPU
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(max(n + 1, 2)), "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 2, r.stderr[-2000:]
    assert "GPU(s) are visible" in r.stderr


def _engine_worker(rank, world, port, outdir):
    """one rank of the sharded run: the HIP engine on its contiguous 8192-gate shard of config 4's
    batch (device 0 for both ranks), gloo for the control plane as bench.py's rehearsal"""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    sys.path.insert(0, gold)
    from fhe_amd import binfhe as bf
    from fhe_amd.dist import barrier, max_over_ranks
    from make_golden import full_inputs
    ps, m, key_seed, keys, bits1, bits2, a1, b1, a2, b2 = full_inputs("std128")
    lo, hi = rank * 8192, (rank + 1) * 8192          # shards 0 and 1 of the 8-GPU split
    eng = bf.GateEngine(ps, m, device=0)
    eng.load_keys(keys.bsk, keys.kskA, keys.kskB)
    barrier()
    ao, bo = eng.eval_gate(1, a1[lo:hi], b1[lo:hi], a2[lo:hi], b2[lo:hi])
    t = max_over_ranks([float(rank + 1)])
    barrier()
    eng.close()
    np.savez(os.path.join(outdir, f"e{rank}.npz"), ao=ao, bo=bo, t=t[0])
    dist.destroy_process_group()


@pytest.mark.gpu
def test_gpu_gloo_world2_engine_shards_bit_exact(tmp_path):
    """two processes, each a GateEngine on its contiguous shard (both on device 0), reassemble to the
    reference's outputs: shard hashes of tests/golden/full_std128.npz"""
    import hashlib
    world = 2
    mp.spawn(_engine_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "full_std128.npz"))
    sha = lambda a: hashlib.sha256(np.ascontiguousarray(a, np.uint64).tobytes()).hexdigest()  # noqa: E731
    for r in range(world):
        p = np.load(tmp_path / f"e{r}.npz")
        assert float(p["t"]) == float(world)
        assert sha(p["ao"]) + sha(p["bo"]) == str(g["shard_sha"][r]), r


def test_bench_reads_the_newest_pmc_summary_in_either_shape(tmp_path, monkeypatch):
    """bench.py's roofline.traffic / valu_busy_pmc come from the newest round's PMC summary, whether it was
    committed in tools/pmc_traffic.py's full form ({"kernels": {...}}) or as its bare kernel map"""
    import glob
    import json
    import bench
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                                          "*pmc_traffic*.json")))
    newest = None
    for f in files:
        d = json.load(open(f))
        ks = d.get("kernels") if isinstance(d.get("kernels"), dict) else d
        if isinstance(ks.get("k_blind_rotate_ginx"), dict):
            newest = ks["k_blind_rotate_ginx"]
    assert newest is not None
    v, b = bench.pmc_summary("k_blind_rotate_ginx", "hbm_bytes_per_launch")
    assert (v, b) == (newest["hbm_bytes_per_launch"], newest["batch"])
    assert bench.pmc_traffic("k_blind_rotate_ginx", b) == newest["hbm_bytes_per_launch"]
    assert bench.pmc_valu_busy("k_blind_rotate_ginx") == newest["valu_busy"]
    # both shapes, the later round winning
    (tmp_path / "profiles").mkdir()
    full = {"round": "r98", "kernels": {"kx": {"batch": 10, "hbm_bytes_per_launch": 100, "valu_busy": 0.5}}}
    bare = {"kx": {"batch": 20, "hbm_bytes_per_launch": 400, "valu_busy": 0.7}}
    json.dump(full, open(tmp_path / "profiles" / "r98_pmc_traffic.json", "w"))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.pmc_summary("kx", "hbm_bytes_per_launch") == (100, 10)
    json.dump(bare, open(tmp_path / "profiles" / "r99_pmc_traffic.json", "w"))
    assert bench.pmc_summary("kx", "hbm_bytes_per_launch") == (400, 20)
    assert bench.pmc_traffic("kx", 40) == 800


def _topology_worker(rank, world, port, outdir):
    """one gloo rank: a device identity (stand-in values: no GPU here) gathered to every rank"""
    import json
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fhe_amd.dist import gather_identities, topology_record
    out = {}
    for case, dev in (("distinct", rank), ("shared", 0)):
        ident = {"rank": rank, "local_rank": rank, "device": dev, "pci": f"0000:{0x10 + dev:02x}:00",
                 "uuid": f"GPU-{dev}", "name": "stand-in", "host": "h0", "peer_access": [True, True]}
        out[case] = topology_record(gather_identities(ident), "gloo", rehearsal=False)
    json.dump(out, open(os.path.join(outdir, f"t{rank}.json"), "w"))
    dist.destroy_process_group()


def test_gloo_world2_bench_topology_record(tmp_path):
    """bench.py's "distributed" object: world size and backend of the process group, every rank's device
    gathered in rank order, distinct-device check; two ranks on one device are a rehearsal, and refused
    under nccl (check_topology)"""
    import json
    from fhe_amd.dist import check_topology
    world = 2
    mp.spawn(_topology_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    recs = [json.load(open(tmp_path / f"t{r}.json")) for r in range(world)]
    assert recs[0] == recs[1]                       # every rank sees the same gathered record
    d, s = recs[0]["distinct"], recs[0]["shared"]
    assert d["world_size"] == 2 and d["backend"] == "gloo" and [i["rank"] for i in d["ranks"]] == [0, 1]
    assert d["distinct_devices"] and d["devices"] == 2 and not d["rehearsal"]
    assert [i["pci"] for i in d["ranks"]] == ["0000:10:00", "0000:11:00"]
    assert not s["distinct_devices"] and s["devices"] == 1 and s["rehearsal"]
    check_topology(d)
    check_topology(s)                                # gloo: a rehearsal is allowed
    with pytest.raises(RuntimeError, match="share a device"):
        check_topology(dict(s, backend="nccl"))
    check_topology(dict(d, backend="nccl"))
