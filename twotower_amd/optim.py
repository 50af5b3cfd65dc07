"""AdamW on the HIP kernels: the same update as torch.optim.AdamW (twotower/train.py:359,
stepped at :139; defaults lr 1e-3, betas (0.9, 0.999), eps 1e-8, weight_decay 1e-2), with the
same per-parameter state keys ('step', 'exp_avg', 'exp_avg_sq') so optimizer state_dicts
interchange.

``fused_tables=True`` lets the embedding tables skip their dense V x E gradient: the bag
backward leaves its factored gradient (ids, d_pooled, denom) on the table and ``step`` runs
the sorted scatter fused with the AdamW update (tt_bag_mean_bwd_adamw).  The result equals the
dense path exactly in math (every row is decayed and its moments updated, rows without tokens
with g = 0), it just never writes or re-reads the dense gradient.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import ops


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 1e-2,
                 fused_tables: bool = False, tables=()):
        if lr < 0.0 or eps < 0.0 or weight_decay < 0.0:
            raise ValueError("invalid AdamW hyper-parameter")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay))
        self._tables: list[torch.Tensor] = []
        if fused_tables:
            ids = {id(p) for g in self.param_groups for p in g["params"]}
            for t in tables:
                inner = getattr(t, "embedding", None)
                w = inner.weight if inner is not None else t
                pad = getattr(inner, "padding_idx", 0) if inner is not None else 0
                if id(w) not in ids:
                    raise ValueError("fused table is not among the optimizer's parameters")
                w._tt_deferred = ops.DeferredTableGrad(pad)
                self._tables.append(w)

    def release_tables(self) -> None:
        """Return the tables to ordinary dense gradients."""
        for w in self._tables:
            if hasattr(w, "_tt_deferred"):
                del w._tt_deferred
        self._tables = []

    def _state(self, p: torch.Tensor) -> dict:
        st = self.state[p]
        if not st:
            st["step"] = torch.tensor(0.0, dtype=torch.float32)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        return st

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            lr, (b1, b2), eps, wd = group["lr"], group["betas"], group["eps"], group["weight_decay"]
            for p in group["params"]:
                deferred = getattr(p, "_tt_deferred", None)
                if deferred is not None and deferred.parts:
                    st = self._state(p)
                    st["step"] += 1
                    ids, dp, den = _merge_parts(deferred.parts)
                    deferred.parts.clear()
                    ops.bag_mean_backward_adamw(dp, den, ids, p.data, st["exp_avg"], st["exp_avg_sq"],
                                                deferred.padding_idx, lr=lr,
                                                beta1=b1, beta2=b2, eps=eps, weight_decay=wd, step=int(st["step"]))
                    continue
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("AdamW does not support sparse gradients")
                st = self._state(p)
                st["step"] += 1
                ops.adamw_step(p.data, p.grad.contiguous(), st["exp_avg"], st["exp_avg_sq"], lr=lr, beta1=b1,
                               beta2=b2, eps=eps, weight_decay=wd, step=int(st["step"]))
        return loss


def _merge_parts(parts):
    if len(parts) == 1:
        return parts[0]
    L = max(ids.shape[1] for ids, _, _ in parts)
    ids = torch.cat([F.pad(i.to(torch.int64), (0, L - i.shape[1])) for i, _, _ in parts], 0)
    return ids, torch.cat([d for _, d, _ in parts], 0), torch.cat([n for _, _, n in parts], 0)
