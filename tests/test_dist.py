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
