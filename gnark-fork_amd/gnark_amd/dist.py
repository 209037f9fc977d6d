"""Multi-GPU MSM sharding over RCCL (one process per GPU, torch.distributed).

The MSM point set shards naturally: rank k keeps the contiguous slice
shard_range(n, k, world) of every key array resident in its own HBM, runs
gg_msm on it and returns a Jacobian partial.  Partials are all-gathered (96 B
per G1 MSM, 192 B per G2) and added on every rank with gg_g1/g2_jac_add --
RCCL has no elliptic-curve reduction op, so this is gather + add, not reduce.
No other data crosses xGMI on the MSM path.
"""
from __future__ import annotations

from . import msm

_JAC = {msm.G1: 96, msm.G2: 192}


def shard_range(n: int, rank: int, world: int):
    """Contiguous, balanced slice [lo, hi) of n points owned by `rank`."""
    lo = n * rank // world
    hi = n * (rank + 1) // world
    return lo, hi


def combine_partials(group: int, partials) -> bytes:
    """Sum of Jacobian partials (bytes) with the library's exact group law."""
    acc = partials[0]
    for p in partials[1:]:
        acc = msm.jac_add(group, acc, p)
    return acc


def allgather_partial(group: int, jac: bytes, device=None) -> bytes:
    """All-gather every rank's partial and return the (identical) sum on all ranks."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    if world == 1:
        return jac
    t = torch.frombuffer(bytearray(jac), dtype=torch.uint8)
    if device is not None:
        t = t.to(device)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return combine_partials(group, [bytes(p.cpu().numpy()) for p in parts])


def group_devices(local_device: int, device=None) -> list:
    """The GPU id of every rank of the process group, in rank order (all-gather)."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return [int(local_device)]
    t = torch.tensor([int(local_device)], dtype=torch.int64)
    if device is not None:
        t = t.to(device)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return [int(p.item()) for p in parts]


def broadcast_bytes(data, nbytes: int, src: int = 0, device=None) -> bytes:
    """`data` (nbytes, significant on rank `src`) on every rank."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return bytes(data)
    if dist.get_rank() == src:
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    else:
        t = torch.zeros(nbytes, dtype=torch.uint8)
    if device is not None:
        t = t.to(device)
    dist.broadcast(t, src)
    return bytes(t.cpu().numpy())
