"""Process-per-GPU helpers for sharded gate batches (bench.py, multi-node-free).

A batch of independent gate bootstraps shards embarrassingly: contiguous
shards, keys replicated, no data-path collective.  The only collectives are
control-plane: a barrier around the timed region and a MAX of the elapsed
times (torch.distributed: "nccl" = RCCL on a GPU box, "gloo" on CPU tests).
"""
import os


def env():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(total, rank, world):
    """Contiguous shard [lo, hi) of `total` items for `rank` (sizes differ by <= 1)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def max_over_ranks(values, device=None):
    """Element-wise MAX of a list of floats over all ranks (identity when not distributed)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [float(v) for v in values]
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.cpu()]


def barrier():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()
