"""Loss registry mirroring twotower/losses.py (contrastive_triplet_loss :9-44,
multiple_negatives_loss :47-85, in_batch_sampled_softmax_loss :88-118, LOSS_REGISTRY :122-127,
build :129-150), every loss on HIP kernels.

The reference training loop always calls ``loss_fn(q, p, n)`` (twotower/train.py:133), which
its own ``multiple_negatives`` / ``in_batch`` entries cannot take.  Here both also accept that
call: ``multiple_negatives`` treats a (B, H) negative as N = 1, and ``in_batch`` scores every
query against all positives and negatives of the batch (candidates = cat[p, n], label of query
i = column i), which is the reference function applied to ``d_emb = cat[p, n]``.  Their
reference signatures keep working unchanged.
"""
from __future__ import annotations

import logging
from functools import partial
from typing import Callable

import torch

from . import ops

logger = logging.getLogger("twotower_amd.losses")


def _packed(*views: torch.Tensor) -> torch.Tensor | None:
    """The common base when the views are consecutive, equally wide row blocks of one contiguous
    2-D tensor in order (TwoTower's fused output split into q, p, n); else None."""
    base = views[0]._base
    if base is None or base.dim() != 2 or not base.is_contiguous():
        return None
    row = base.shape[1] * base.element_size()
    at = base.data_ptr()
    for v in views:
        if v._base is not base or v.dim() != 2 or not v.is_contiguous() or v.shape[1] != base.shape[1]:
            return None
        if v.data_ptr() != at:
            return None
        at += v.shape[0] * row
    if at != base.data_ptr() + base.shape[0] * row:
        return None
    return base


def contrastive_triplet_loss(q_emb: torch.Tensor, d_pos_emb: torch.Tensor, d_neg_emb: torch.Tensor,
                             margin: float = 0.2) -> torch.Tensor:
    """mean(relu(margin - cos(q, d+) + cos(q, d-))) (losses.py:9-44)."""
    base = _packed(q_emb, d_pos_emb, d_neg_emb)
    if base is not None and q_emb.shape[0] == d_pos_emb.shape[0] == d_neg_emb.shape[0]:
        return ops.TripletLossPacked.apply(base, margin)
    return ops.TripletLoss.apply(q_emb, d_pos_emb, d_neg_emb, margin)


def multiple_negatives_loss(q_emb: torch.Tensor, d_pos_emb: torch.Tensor, d_neg_embs: torch.Tensor,
                            temperature: float = 0.1) -> torch.Tensor:
    """InfoNCE over [d+, d-_1..N] by cosine / temperature, label 0 (losses.py:47-85)."""
    if d_neg_embs.dim() == 2:
        d_neg_embs = d_neg_embs.unsqueeze(1)
    B, K = d_neg_embs.shape[0], d_neg_embs.shape[1]
    if d_neg_embs.is_contiguous() and d_pos_emb.shape[0] == q_emb.shape[0] == B:
        base = _packed(q_emb, d_pos_emb, d_neg_embs.view(B * K, -1))
        if base is not None:  # [q; p; negatives] in one tensor (TwoTower's fused output): one gradient tensor
            return ops.MultiNegLossPacked.apply(base, B, K, 1.0 / float(temperature))
    return ops.MultiNegLoss.apply(q_emb, d_pos_emb, d_neg_embs, 1.0 / float(temperature))


def _candidates(p: torch.Tensor, n: torch.Tensor) -> torch.Tensor:
    """cat([p, n]) without a copy when p and n are consecutive row blocks of one tensor
    (TwoTower's fused output): a narrow() of their common base, so autograd stays exact."""
    base = p._base
    if (base is not None and base is n._base and base.dim() == 2 and base.is_contiguous() and p.dim() == 2
            and p.is_contiguous() and n.is_contiguous() and p.shape[1] == base.shape[1] == n.shape[1]):
        row = base.shape[1] * base.element_size()
        start = (p.data_ptr() - base.data_ptr()) // row
        if (p.data_ptr() - base.data_ptr()) % row == 0 and n.data_ptr() == p.data_ptr() + p.shape[0] * row:
            return base.narrow(0, start, p.shape[0] + n.shape[0])
    return torch.cat([p, n], dim=0)


def in_batch_sampled_softmax_loss(q_emb: torch.Tensor, d_emb: torch.Tensor, *args, temperature: float = 0.1,
                                  compute_dtype: str = "fp32", cross_device_negatives: bool = False,
                                  group=None) -> torch.Tensor:
    """CE over S = q d^T / temperature with labels arange(B) (losses.py:88-118), on the fused
    MFMA scorer.  Third positional argument: a negatives tensor (train.py:133 call) or the
    reference's positional temperature.  ``cross_device_negatives`` scores every data-parallel
    rank's candidates (RCCL all-gather, labels offset by this rank's slot); at bf16 each rank
    then computes the gradient of its own candidates (ops.InBatchSoftmaxLossOwned)."""
    if args:
        if isinstance(args[0], torch.Tensor):
            if len(args) > 1:
                temperature = args[1]
            base = None if cross_device_negatives else _packed(q_emb, d_emb, args[0])
            if base is not None:  # [q; p; n] in one tensor: zero-copy candidates and gradient
                return ops.InBatchSoftmaxLossPacked.apply(base, q_emb.shape[0], 1.0 / float(temperature),
                                                          compute_dtype, None)
            d_emb = _candidates(d_emb, args[0])
        else:
            temperature = args[0]
    if not cross_device_negatives and (not args or not isinstance(args[0], torch.Tensor)):
        base = _packed(q_emb, d_emb)
        if base is not None:  # (query, positive) pairs as [q; d] in one tensor (TwoTower(q, d)): the
            # same packed path, so the head's operand prep and fused L2 backward apply to M = B too
            return ops.InBatchSoftmaxLossPacked.apply(base, q_emb.shape[0], 1.0 / float(temperature),
                                                      compute_dtype, None)
    label_off = 0
    if cross_device_negatives:
        from . import distributed

        if (distributed.is_active(group) and compute_dtype != "fp32" and _owner_gradients()):
            # bf16 candidate copies all-gathered, candidate gradients computed by their owners
            return ops.InBatchSoftmaxLossOwned.apply(q_emb, d_emb, 1.0 / float(temperature), compute_dtype, None,
                                                     group)
        d_emb, label_off = distributed.gather_candidates(d_emb, group=group)
    return ops.in_batch_softmax_loss(q_emb, d_emb, temperature, label_off=label_off, compute_dtype=compute_dtype)


def scorer_prep_dtype(loss_fn) -> str | None:
    """The compute dtype when ``loss_fn`` is a single-device in-batch loss (as built by
    ``build("in_batch", compute_dtype=..., ...)``), whose operand prep a tied TwoTower may fold
    into its head's normalise pass (ops.scorer_prep; the head fuses it where tt_inbatch_l2_prep
    has the shape: bf16 / bf16_split at H = 256, fp32 at H = 128); else None."""
    fn, kw = (loss_fn.func, loss_fn.keywords) if isinstance(loss_fn, partial) else (loss_fn, {})
    if fn is not in_batch_sampled_softmax_loss or kw.get("cross_device_negatives"):
        return None
    dt = kw.get("compute_dtype", "fp32")
    return dt if dt in ("bf16", "bf16_split", "fp32") else None


def _owner_gradients() -> bool:
    """Cross-device negatives at bf16: candidate-owner gradients (default) or TT_INBATCH_DP=
    allgather for the fp32-row all-gather + gradient reduce-scatter form (the fp32 path)."""
    import os

    return os.environ.get("TT_INBATCH_DP", "owner") != "allgather"


LOSS_REGISTRY = {
    "triplet": contrastive_triplet_loss,
    "multiple_negatives": multiple_negatives_loss,
    "in_batch": in_batch_sampled_softmax_loss,
}


def build(name: str, **kwargs) -> Callable:
    """Loss by name with bound kwargs (losses.py:129-150)."""
    if name not in LOSS_REGISTRY:
        raise ValueError(f"Unknown loss function: {name}. Available options: {list(LOSS_REGISTRY.keys())}")
    fn = LOSS_REGISTRY[name]
    return partial(fn, **kwargs) if kwargs else fn
