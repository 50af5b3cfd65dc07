"""Tower registry and TwoTower, mirroring twotower/encoders.py (BaseTower :12-22,
MeanPoolingTower :25-81, AveragePoolingTower :84-155, TwoTower :158-224, TOWER_REGISTRY
:228-232, build_tower :234-249, build_two_tower :251-272).

Parameter names match the reference (`embedding.embedding.weight`, `feed_forward.{0,2}.*`,
`projection.{0,2}.*`) so state_dicts load in either direction.  The pooled lookup runs on the
fused HIP bag kernel; TwoTower.forward pools the query, positive and negative ids of a step in
ONE launch over the shared table (the towers always share it, encoders.py:265,270).
"""
from __future__ import annotations

import contextlib
import logging

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .embeddings import BaseEmbedding

logger = logging.getLogger("twotower_amd.encoders")


def pool_mean(embedding: nn.Module, input_ids: torch.Tensor) -> torch.Tensor:
    """Fused gather + masked mean (encoders.py:62-72).  Accepts this package's embeddings and
    any reference-style embedding that holds an nn.Embedding at `.embedding`."""
    if hasattr(embedding, "pool_mean"):
        return embedding.pool_mean(input_ids)
    inner = getattr(embedding, "embedding", None)
    if isinstance(inner, nn.Embedding):
        return ops.bag_mean_pool(inner.weight, input_ids, inner.padding_idx)
    raise TypeError(f"{type(embedding).__name__} exposes no lookup table for the fused bag kernel")


def _table_of(embedding: nn.Module) -> torch.Tensor | None:
    inner = getattr(embedding, "embedding", None)
    return inner.weight if isinstance(inner, nn.Embedding) else None


def _planes_in_gather(tower: nn.Module, ids: torch.Tensor):
    """The gather feeding this tower's hand-written head also forms the head's weight planes
    (ops.head_planes_in_gather)."""
    if ids.is_cuda and type(tower).encode_pooled is MeanPoolingTower.encode_pooled:
        ff = tower._layers()
        if tower.hand_written_head(ff):
            return ops.head_planes_in_gather(ff[0].weight, ff[2].weight)
    return contextlib.nullcontext()


def _sole_head(tower: nn.Module, pooled: torch.Tensor):
    """The pooled rows go to this tower's own fused head and nowhere else (MeanPoolingTower's
    encode_pooled, not overridden): its backward may then hand the bag backward d_pooled / denom
    (ops.bag_head_prescale)."""
    if type(tower).encode_pooled is MeanPoolingTower.encode_pooled:
        return ops.bag_head_prescale(pooled)
    return contextlib.nullcontext()


class BaseTower(nn.Module):
    """Base class for tower/encoder architectures (encoders.py:12-22)."""

    def __init__(self, embedding: BaseEmbedding, hidden_dim: int):
        super().__init__()
        self.embedding = embedding
        self.hidden_dim = hidden_dim

    def log_params(self):
        n = sum(p.numel() for p in self.parameters() if p.requires_grad)
        logger.info(f"Tower parameters: {n:,}")

    def encode_pooled(self, pooled: torch.Tensor) -> torch.Tensor:  # pragma: no cover - abstract
        raise NotImplementedError

    def forward(self, input_ids: torch.Tensor) -> torch.Tensor:
        with _planes_in_gather(self, input_ids):
            pooled = pool_mean(self.embedding, input_ids)
            with _sole_head(self, pooled):
                return self.encode_pooled(pooled)


class MeanPoolingTower(BaseTower):
    """Masked mean-pool -> Linear-ReLU-Linear -> L2 normalise (encoders.py:25-81)."""

    def __init__(self, embedding: BaseEmbedding, hidden_dim: int):
        super().__init__(embedding, hidden_dim)
        embedding_dim = embedding.embedding_dim
        self.feed_forward = nn.Sequential(
            nn.Linear(embedding_dim, hidden_dim),
            nn.ReLU(),
            nn.Linear(hidden_dim, hidden_dim),
        )
        self.log_params()

    def _layers(self) -> tuple:
        """feed_forward's modules (one dict read: nn.Sequential indexing costs a few us per item,
        and the fused forward asks for the layers a dozen times per step)."""
        ff = self.feed_forward
        return tuple(ff._modules.values()) if isinstance(ff, nn.Sequential) else ()

    def _standard_ff(self, ff: tuple | None = None) -> bool:
        ff = self._layers() if ff is None else ff
        return (len(ff) == 3 and isinstance(ff[0], nn.Linear) and isinstance(ff[1], nn.ReLU)
                and isinstance(ff[2], nn.Linear) and ff[0].bias is not None and ff[2].bias is not None)

    def hand_written_head(self, ff: tuple | None = None) -> bool:
        """The head runs on ops.tower_head (the hand-written split-bf16 GEMMs)."""
        ff = self._layers() if ff is None else ff
        return (self._standard_ff(ff) and ff[0].out_features == ff[2].out_features == ff[2].in_features
                in ops.HEAD_WIDTHS and ff[0].in_features in ops.EMB_WIDTHS)

    def encode_pooled(self, pooled: torch.Tensor) -> torch.Tensor:
        ff = self._layers()
        if self.hand_written_head(ff):
            # Linear-ReLU-Linear + F.normalize in two fused GEMM launches (encoders.py:38-42,77)
            return ops.tower_head(pooled.contiguous(), ff[0].weight, ff[0].bias, ff[2].weight, ff[2].bias)
        if self._standard_ff(ff) and ff[0].out_features % 4 == 0 and ff[2].out_features % 4 == 0:
            y = ops.tower_ff(pooled.contiguous(), ff[0].weight, ff[0].bias, ff[2].weight, ff[2].bias)
        else:  # a user-modified head (or widths off the vec4 column-sum): run it as given
            y = self.feed_forward(pooled)
        return ops.l2_normalize(y)  # encoders.py:77


class AveragePoolingTower(BaseTower):
    """Masked mean-pool -> optional Linear-Dropout-LayerNorm -> L2 normalise (encoders.py:84-155)."""

    def __init__(self, embedding: BaseEmbedding, hidden_dim: int, dropout: float = 0.1):
        super().__init__(embedding, hidden_dim)
        embedding_dim = embedding.embedding_dim
        self.has_projection = hidden_dim != embedding_dim
        if self.has_projection:
            self.projection = nn.Sequential(
                nn.Linear(embedding_dim, hidden_dim),
                nn.Dropout(dropout),
                nn.LayerNorm(hidden_dim),
            )
        self.log_params()

    def encode_pooled(self, pooled: torch.Tensor) -> torch.Tensor:
        if not self.has_projection:
            return ops.l2_normalize(pooled.contiguous())  # encoders.py:150
        lin, drop, ln = self.projection
        if (isinstance(lin, nn.Linear) and isinstance(drop, nn.Dropout) and isinstance(ln, nn.LayerNorm)
                and ln.elementwise_affine and ln.weight.shape[0] % 4 == 0):
            if (pooled.is_cuda and lin.bias is not None
                    and ops.linear_widths_ok(lin.in_features, lin.out_features)):
                h = ops.linear(pooled.contiguous(), lin.weight, lin.bias)  # split-bf16 MFMA Linear
            else:  # widths outside the hand-written kernels: the library GEMM
                h = F.linear(pooled, lin.weight, lin.bias)
            h = F.dropout(h, drop.p, self.training)
            return ops.layernorm_l2_normalize(h, ln.weight, ln.bias, ln.eps)  # one fused row pass
        return ops.l2_normalize(self.projection(pooled).contiguous())


def _packed_ids(inputs: list[torch.Tensor]) -> torch.Tensor | None:
    """The common (N, L) base when the id tensors are consecutive row blocks of it in order
    (TrainStep's packed static batch), so the fused forward needs no concatenation."""
    base = inputs[0]._base
    if base is None or base.dim() != 2 or not base.is_contiguous():
        return None
    at, row = base.data_ptr(), base.shape[1] * base.element_size()
    for t in inputs:
        if t._base is not base or not t.is_contiguous() or t.shape[1] != base.shape[1] or t.data_ptr() != at:
            return None
        at += t.shape[0] * row
    return base if at == base.data_ptr() + base.shape[0] * row else None


class TwoTower(nn.Module):
    """Query and document towers (encoders.py:158-224)."""

    def __init__(self, query_tower: BaseTower, document_tower: BaseTower | None = None, tied_weights: bool = False):
        super().__init__()
        self.query_tower = query_tower
        if tied_weights:
            self.document_tower = query_tower
        else:
            self.document_tower = document_tower if document_tower is not None else query_tower
        # compute dtype of an in-batch loss whose operand prep the fused forward may fold into the
        # tower head's normalise pass (ops.scorer_prep; TrainStep sets it); None: never
        self.scorer_prep: str | None = None
        total = sum(p.numel() for p in self.parameters() if p.requires_grad)
        logger.info(f"Total trainable parameters: {total:,}")

    def _fusable(self) -> bool:
        qt, dt = self.query_tower, self.document_tower
        if not (isinstance(qt, BaseTower) and isinstance(dt, BaseTower)):
            return False
        tq, td = _table_of(qt.embedding), _table_of(dt.embedding)
        return tq is not None and tq is td

    def forward(self, query_input, document_input=None, negative_input=None):
        inputs = [t for t in (query_input, document_input, negative_input) if t is not None]
        if len(inputs) > 1 and self._fusable():
            outs = self._forward_fused(inputs)
        else:
            outs = [self.query_tower(query_input)]
            outs += [self.document_tower(t) for t in inputs[1:]]
        return outs[0] if len(outs) == 1 else tuple(outs)

    def _forward_fused(self, inputs: list[torch.Tensor]) -> list[torch.Tensor]:
        """One bag launch over all sequences of the step, then the towers' heads."""
        all_ids = _packed_ids(inputs)
        if all_ids is None:
            L = max(t.shape[1] for t in inputs)
            ids = [t if t.shape[1] == L else F.pad(t, (0, L - t.shape[1])) for t in inputs]
            dtype = torch.int64 if any(t.dtype == torch.int64 for t in ids) else ids[0].dtype
            all_ids = torch.cat([t.to(dtype) for t in ids], dim=0)
        sizes = [t.shape[0] for t in inputs]
        nq = sizes[0]
        if self.query_tower is self.document_tower:
            with _planes_in_gather(self.query_tower, all_ids):
                pooled = pool_mean(self.query_tower.embedding, all_ids)
                prep = ops.scorer_prep(nq, self.scorer_prep) if self.scorer_prep else contextlib.nullcontext()
                with prep, _sole_head(self.query_tower, pooled):
                    # one head over all rows: its normalise pass may also prep the in-batch scorer
                    return list(torch.split(self.query_tower.encode_pooled(pooled), sizes, dim=0))
        pooled = pool_mean(self.query_tower.embedding, all_ids)
        q = self.query_tower.encode_pooled(pooled[:nq])
        docs = self.document_tower.encode_pooled(pooled[nq:])
        return [q] + list(torch.split(docs, sizes[1:], dim=0))

    def encode_query(self, query_input):
        return self.query_tower(query_input)

    def encode_document(self, document_input):
        return self.document_tower(document_input)


TOWER_REGISTRY = {
    "mean": MeanPoolingTower,
    "avg_pool": AveragePoolingTower,
}


def build_tower(name: str, embedding: BaseEmbedding, **kwargs) -> BaseTower:
    """Build a tower by name (encoders.py:234-249)."""
    if name not in TOWER_REGISTRY:
        raise ValueError(f"Unknown tower architecture: {name}. Available options: {list(TOWER_REGISTRY.keys())}")
    return TOWER_REGISTRY[name](embedding=embedding, **kwargs)


def build_two_tower(tower_name: str, embedding: BaseEmbedding, hidden_dim: int, tied_weights: bool = False,
                    **kwargs) -> TwoTower:
    """Build a complete two-tower model (encoders.py:251-272)."""
    query_tower = build_tower(tower_name, embedding, hidden_dim=hidden_dim, **kwargs)
    document_tower = None if tied_weights else build_tower(tower_name, embedding, hidden_dim=hidden_dim, **kwargs)
    return TwoTower(query_tower, document_tower, tied_weights=tied_weights)
