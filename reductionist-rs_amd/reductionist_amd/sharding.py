"""Multi-GPU placement for independent chunks: one process per GPU, each owning a
disjoint subset of the chunks; no data-path collective (a request's result depends on its chunk
only).  The control plane (barrier, max-over-ranks timing) uses torch.distributed on the host."""
from __future__ import annotations

import os


def rank_info():
    """(rank, world, local_rank) from the torchrun environment (1-process defaults)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_range(n_items: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, balanced split of [0, n_items): sizes differ by at most one."""
    base, extra = divmod(n_items, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def device_for(local_rank: int, n_devices: int) -> int:
    """GPU of a rank (several ranks may share a device when rehearsing on fewer GPUs)."""
    if n_devices <= 0:
        raise RuntimeError("no device")
    return local_rank % n_devices


def max_over_ranks(x: float) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0])


def barrier() -> None:
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()
