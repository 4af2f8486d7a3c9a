"""Multi-GPU sharding of a chunk batch.

Chunks are independent, so a batch shards round-robin over the GPUs of a node
(chunk i -> rank i mod world), one process per GPU, with NO collective on the
data path: each rank CRCs its own chunks in its own HBM.  Only the 4-byte
results travel, and only when a caller wants the whole batch's results on one
rank (gather_results), e.g. to write chunk headers or verify a scan.
"""
import numpy as np


def shard_ids(n, rank, world):
    """Chunk indices owned by `rank` (round-robin)."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    return np.arange(rank, n, world, dtype=np.int64)


def assemble(n, world, parts):
    """Scatter per-rank result arrays (in shard order) back to batch order."""
    out = np.empty(n, dtype=np.uint32)
    for r, p in enumerate(parts):
        ids = shard_ids(n, r, world)
        if len(p) != len(ids):
            raise ValueError(f"rank {r}: {len(p)} results for {len(ids)} chunks")
        out[ids] = p
    return out


def gather_results(local, n, group=None, dst=None):
    """Collect every rank's uint32 results into batch order.

    Uses torch.distributed (gloo on CPU tensors, or RCCL on cuda tensors);
    returns the full array on every rank (dst=None) or only on `dst`.
    """
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    maxlen = (n + world - 1) // world
    dev = local.device if isinstance(local, torch.Tensor) else torch.device("cpu")
    buf = torch.zeros(maxlen, dtype=torch.int64, device=dev)
    loc = local if isinstance(local, torch.Tensor) else torch.from_numpy(
        np.asarray(local, dtype=np.uint32).astype(np.int64))
    buf[: len(loc)] = loc.to(dev).to(torch.int64)
    if dst is None:
        bufs = [torch.zeros_like(buf) for _ in range(world)]
        dist.all_gather(bufs, buf, group=group)
    else:
        bufs = [torch.zeros_like(buf) for _ in range(world)] if rank == dst else None
        dist.gather(buf, bufs, dst=dst, group=group)
        if rank != dst:
            return None
    parts = [b.cpu().numpy()[: len(shard_ids(n, r, world))].astype(np.uint32) for r, b in enumerate(bufs)]
    return assemble(n, world, parts)
