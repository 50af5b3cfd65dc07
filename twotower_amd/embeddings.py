"""Embedding registry, mirroring twotower/embeddings.py (BaseEmbedding :10-21,
LookupEmbedding :24-40, REGISTRY :159-164, build :166-181).

`LookupEmbedding` keeps the reference's parameter layout (submodule `.embedding` holding an
nn.Embedding(V, E, padding_idx=0) weight, same init) so state_dicts interchange, and adds
`pool_mean(ids)`: the fused HIP gather + masked mean-pool that the towers call instead of
materialising the (B, L, E) lookup.
"""
from __future__ import annotations

import logging
from abc import ABC

import torch
import torch.nn as nn

from . import _lib, ops

logger = logging.getLogger("twotower_amd.embeddings")


class BaseEmbedding(nn.Module, ABC):
    """Base class for all embedding layers (twotower/embeddings.py:10-21)."""

    def __init__(self, vocab_size: int, embedding_dim: int, padding_idx: int = 0):
        super().__init__()
        self.vocab_size = vocab_size
        self.embedding_dim = embedding_dim
        self.padding_idx = padding_idx

    def log_params(self):
        logger.info(f"Embedding parameters: {self.vocab_size * self.embedding_dim:,}")


class LookupEmbedding(BaseEmbedding):
    """Trainable lookup table (twotower/embeddings.py:24-40) with a fused pooled lookup."""

    def __init__(self, vocab_size: int, embedding_dim: int, padding_idx: int = 0,
                 scatter_mode: str = "sorted"):
        super().__init__(vocab_size, embedding_dim, padding_idx)
        self.embedding = nn.Embedding(vocab_size, embedding_dim, padding_idx=padding_idx)
        if scatter_mode not in ("sorted", "atomic"):
            raise ValueError(f"scatter_mode must be 'sorted' or 'atomic', got {scatter_mode!r}")
        self.scatter_mode = scatter_mode
        self.log_params()

    @property
    def weight(self) -> torch.Tensor:
        return self.embedding.weight

    def forward(self, input_ids: torch.Tensor) -> torch.Tensor:
        """(B, L) ids -> (B, L, E) rows: the reference's unfused contract, kept for foreign
        towers.  The towers of this package never call it (they use pool_mean)."""
        return self.embedding(input_ids)

    def pool_mean(self, input_ids: torch.Tensor) -> torch.Tensor:
        """(B, L) ids -> (B, E): sum_{ids>0} W[ids] / (count + 1e-9) on the HIP bag kernel
        (twotower/encoders.py:62-72 fused with the lookup at embeddings.py:40)."""
        mode = _lib.TT_SCATTER_SORTED if self.scatter_mode == "sorted" else _lib.TT_SCATTER_ATOMIC
        return ops.bag_mean_pool(self.embedding.weight, input_ids, self.padding_idx, mode)


class _Unavailable(BaseEmbedding):
    """word2vec / glove need gensim and a network download (embeddings.py:49,101,107); neither
    exists in this environment, and both are outside the accelerated path."""

    def __init__(self, *args, **kwargs):
        raise ImportError(f"{type(self).__name__}: pretrained vectors need gensim + network access; "
                          "not provided by twotower_amd")


class FrozenWord2Vec(_Unavailable):
    pass


class GloVeEmbedding(_Unavailable):
    pass


REGISTRY = {
    "lookup": LookupEmbedding,
    "word2vec": FrozenWord2Vec,
    "glove": GloVeEmbedding,
}


def build(name: str, vocab_size: int, **kwargs) -> BaseEmbedding:
    """Build an embedding layer by name (twotower/embeddings.py:166-181)."""
    if name not in REGISTRY:
        raise ValueError(f"Unknown embedding: {name}. Available options: {list(REGISTRY.keys())}")
    return REGISTRY[name](vocab_size=vocab_size, **kwargs)
