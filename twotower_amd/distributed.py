"""Data parallelism for the two-tower step: one process per GPU, torch.distributed over RCCL
(backend "nccl" on ROCm) across xGMI; gloo for the CPU tests of the same logic.

The reference has no distributed code.  This module adds exactly the exchanges
the step needs:
  * in-batch negatives: the candidate embeddings of every rank are all-gathered (rank-major),
    rank r's labels are offset by r * local_M, and the gather's backward reduce-scatters the
    candidate gradients back to their owners;
  * gradient sync: the loss is pre-scaled by 1/world so one SUM all-reduce per bucket yields the
    global-batch mean gradient (no separate averaging pass over the 205 MB table gradient).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def is_active(group=None) -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1


class AllGatherRows(torch.autograd.Function):
    """out = cat over ranks of x (rank-major); backward = reduce_scatter(SUM) of the gradient."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        world = dist.get_world_size(group)
        x = x.contiguous()
        out = x.new_empty((world * x.shape[0],) + tuple(x.shape[1:]))
        dist.all_gather_into_tensor(out, x, group=group)
        return out

    @staticmethod
    def backward(ctx, g):
        world = dist.get_world_size(ctx.group)
        g = g.contiguous()
        out = g.new_empty((g.shape[0] // world,) + tuple(g.shape[1:]))
        dist.reduce_scatter_tensor(out, g, op=dist.ReduceOp.SUM, group=ctx.group)
        return out, None


def gather_candidates(d: torch.Tensor, group=None) -> tuple[torch.Tensor, int]:
    """All ranks' candidate rows and this rank's label offset (its first candidate row)."""
    if not is_active(group):
        return d, 0
    return AllGatherRows.apply(d, group), dist.get_rank(group) * d.shape[0]


class GradSync:
    """Sum-all-reduce of every gradient after backward.  Small parameters travel in one flat
    bucket; large ones (the embedding table) are reduced in place.  With the loss pre-scaled
    by 1/world the sums are the global-batch mean gradients."""

    def __init__(self, params, group=None, bucket_cap: int = 1 << 22):
        self.group = group
        self.params = [p for p in params if p.requires_grad]
        self.bucket_cap = bucket_cap

    @property
    def world(self) -> int:
        return dist.get_world_size(self.group) if is_active(self.group) else 1

    def loss_scale(self) -> float:
        return 1.0 / self.world

    def sync(self) -> None:
        if not is_active(self.group):
            return
        small = [p for p in self.params if p.grad is not None and p.numel() <= self.bucket_cap]
        large = [p for p in self.params if p.grad is not None and p.numel() > self.bucket_cap]
        works = []
        if small:
            flat = torch.cat([p.grad.reshape(-1) for p in small])
            works.append((dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True), flat, small))
        for p in large:
            works.append((dist.all_reduce(p.grad, op=dist.ReduceOp.SUM, group=self.group, async_op=True), None, None))
        for work, flat, members in works:
            work.wait()
            if flat is not None:
                off = 0
                for p in members:
                    n = p.numel()
                    p.grad.copy_(flat[off:off + n].view_as(p.grad))
                    off += n
