"""Batch sharding across ranks (one process per GPU) and the optional RCCL all-gather of outputs.

KDLAE-T images are independent units (MDTA reduces only within an image, KDLAE_model.py:130-140),
so a global batch B is split contiguously: rank r owns images [r*B/N, (r+1)*B/N).  There is no
collective on the data path; ``gather_outputs`` is the optional all-gather (RCCL over xGMI via the
torch ``nccl`` backend) for callers that need the whole batch on every rank.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n_items: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, rank-ordered split; sizes differ by at most one item."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    base, extra = divmod(n_items, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard_batch(batch: dict, rank: int, world: int) -> dict:
    """Slice every tensor of a KDLAE-T input dict ({'img', 'denoise_rate'}) to this rank's images."""
    n = next(iter(batch.values())).shape[0]
    s, e = shard_range(n, rank, world)
    return {k: v[s:e] for k, v in batch.items()}


def gather_outputs(local: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather equal-sized per-rank shards into the full batch in rank order."""
    world = dist.get_world_size(group)
    out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    if hasattr(dist, "all_gather_into_tensor") and dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    else:
        dist.all_gather(list(out.chunk(world)), local.contiguous(), group=group)
    return out


def sharded_forward(model, batch: dict, group=None, gather: bool = True) -> dict:
    """Run this rank's shard of ``batch`` through ``model``; optionally all-gather hq / sr.

    The global batch must divide evenly across ranks when ``gather`` is set (equal shard sizes).
    """
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    n = next(iter(batch.values())).shape[0]
    if gather and n % world:
        raise ValueError(f"global batch {n} must be divisible by world size {world} to gather")
    out = model(shard_batch(batch, rank, world))
    if not gather:
        return out
    return {k: (gather_outputs(v, group) if v is not None else None) for k, v in out.items()}
