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


def _batch_size(batch: dict) -> int:
    if batch.get("img") is not None:
        return batch["img"].shape[0]
    for v in batch.values():
        if v is not None:
            return v.shape[0]
    raise ValueError("empty batch")


def shard_batch(batch: dict, rank: int, world: int) -> dict:
    """Slice every tensor of a KDLAE-T input dict ({'img', 'denoise_rate'}) to this rank's images;
    None entries (``denoise_rate`` when params != 'cat') pass through."""
    s, e = shard_range(_batch_size(batch), rank, world)
    return {k: (v[s:e] if v is not None else None) for k, v in batch.items()}


def gather_outputs(local: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather equal-sized per-rank shards into the full batch in rank order."""
    world = dist.get_world_size(group)
    if local.is_cuda and dist.get_backend(group) != "nccl":
        # gloo moves host memory: stage a device shard through the host (multi-process tests on one GPU)
        return gather_outputs(local.cpu(), group).to(local.device)
    out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    if hasattr(dist, "all_gather_into_tensor") and dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    else:
        dist.all_gather(list(out.chunk(world)), local.contiguous(), group=group)
    return out


def gather_outputs_async(local: torch.Tensor, group=None):
    """Start the all-gather of equal-sized per-rank shards and return ``(full, work)`` without
    waiting: ``full`` holds the batch in rank order once ``work`` has completed.  RCCL (nccl) runs
    it on its own stream behind the caller's current point, so the caller's next kernels overlap
    it; ``work.wait()`` orders the caller's stream after it (gloo: blocks the host until done).
    A device tensor under gloo is staged through the host synchronously (``work`` None)."""
    world = dist.get_world_size(group)
    backend = dist.get_backend(group)
    if (local.is_cuda and backend != "nccl") or not hasattr(dist, "all_gather_into_tensor"):
        return gather_outputs(local, group), None
    out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    work = dist.all_gather_into_tensor(out, local.contiguous(), group=group, async_op=True)
    return out, work


class OverlappedGather:
    """The SURVEY §8e output all-gather with step i's gather overlapping step i + 1's forward:
    each step enqueues its hq / sr gathers asynchronously (RCCL's own stream,
    gather_outputs_async), at most `depth` steps stay in flight (the oldest is waited for first),
    and drain() orders the caller's stream after the rest.  A step's returned tensors are complete
    once its gathers are: bench.py's timed_steps drains inside the timed window, so every step's
    gather is counted, and the last step's output is read only after that."""

    def __init__(self, depth: int = 2, group=None):
        self.depth = depth
        self.group = group
        self.inflight = []

    def __call__(self, out: dict) -> dict:
        res, works = {}, []
        for k, v in out.items():
            if v is None:
                res[k] = None
                continue
            res[k], work = gather_outputs_async(v, self.group)
            if work is not None:
                works.append(work)
        self.inflight.append(works)
        while len(self.inflight) > self.depth:
            for w in self.inflight.pop(0):
                w.wait()
        return res

    def drain(self):
        while self.inflight:
            for w in self.inflight.pop(0):
                w.wait()


def sharded_forward(model, batch: dict, group=None, gather: bool = True) -> dict:
    """Run this rank's shard of ``batch`` through ``model``; optionally all-gather hq / sr.

    The global batch must divide evenly across ranks when ``gather`` is set (equal shard sizes).
    """
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    n = _batch_size(batch)
    if gather and n % world:
        raise ValueError(f"global batch {n} must be divisible by world size {world} to gather")
    out = model(shard_batch(batch, rank, world))
    if not gather:
        return out
    return {k: (gather_outputs(v, group) if v is not None else None) for k, v in out.items()}


def gather_varlen(local: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather shards whose leading sizes differ by rank (a contiguous split of N items that
    does not divide evenly): pad to the largest shard, gather, trim, concatenate in rank order."""
    world = dist.get_world_size(group)
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(x.item()) for x in sizes]
    m = max(sizes)
    padded = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    padded[:local.shape[0]] = local
    full = gather_outputs(padded, group)
    return torch.cat([full[r * m:r * m + sizes[r]] for r in range(world)])


def sharded_scores(model, lq: torch.Tensor, gt: torch.Tensor, group=None, gather: bool = True,
                   chunk: int = 64) -> torch.Tensor:
    """ASDQE batch scoring (ASDQE/ASDQE_test.py:87-104 ``infer``) split across ranks: rank r scores
    its contiguous share of the N (lq, gt) pairs in chunks of ``chunk`` images, then (``gather``)
    the [N, 1] scores are all-gathered in rank order, so every rank holds the full score list."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    s, e = shard_range(lq.shape[0], rank, world)
    dev = next(model.parameters()).device
    parts = []
    with torch.no_grad():
        for c0 in range(s, e, chunk):
            c1 = min(e, c0 + chunk)
            parts.append(model(lq[c0:c1].to(dev), gt[c0:c1].to(dev)).reshape(-1, 1))
    local = torch.cat(parts) if parts else torch.zeros((0, 1), device=dev)
    return gather_varlen(local, group) if gather else local
