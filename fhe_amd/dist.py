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


def device_identity(torch, dev, rank, local):
    """This rank's device as the N-rank bench line records it: index, PCI address, UUID, name, host, and
    which visible devices it can reach by peer access (hipDeviceCanAccessPeer: the MultiEngine key
    fan-out copies device 0's packed keys to every other device)."""
    import socket
    p = torch.cuda.get_device_properties(dev)
    n = torch.cuda.device_count()
    return {"rank": rank, "local_rank": local, "device": dev.index,
            "pci": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}",
            "uuid": str(getattr(p, "uuid", "")), "name": p.name, "host": socket.gethostname(),
            "peer_access": [bool(j == dev.index or torch.cuda.can_device_access_peer(dev.index, j)) for j in range(n)]}


def gather_identities(ident):
    """every rank's identity (device_identity) in rank order, on every rank; one process: [ident]"""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [ident]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, ident)
    return out


def topology_record(idents, backend, rehearsal):
    """The "distributed" object of the bench line: the process group's world size and backend as the
    ranks saw them, each rank's device, and whether the ranks ran on distinct devices (host, PCI address,
    UUID).  A run whose ranks share a device is a rehearsal (FHE_BENCH_DEVICE_MAP / gloo on one GPU), not a
    scaling measurement; check_topology refuses it under RCCL."""
    keys = [(i["host"], i["pci"], i["uuid"]) for i in idents]
    distinct = len(set(keys)) == len(keys)
    return {"world_size": len(idents), "backend": backend, "ranks": idents, "distinct_devices": distinct,
            "devices": len(set(keys)), "rehearsal": bool(rehearsal) or not distinct,
            "note": "rehearsal: several ranks on one GPU, not a scaling number" if (rehearsal or not distinct)
                    else "one rank per distinct GPU"}


def check_topology(rec):
    """RCCL ranks must each own a GPU: raise when two "nccl" ranks report the same device"""
    if rec["backend"] == "nccl" and rec["world_size"] > 1 and not rec["distinct_devices"]:
        dup = [(i["rank"], i["pci"]) for i in rec["ranks"]]
        raise RuntimeError(f"nccl ranks share a device: {dup}")
