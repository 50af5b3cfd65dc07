"""twotower_amd — MI355X (gfx950) two-tower training step behind the reference's plugin surface.

Public surface mirrors k0r1g/two-towers' ``twotower`` package for the accelerated path:
``embeddings.{BaseEmbedding, LookupEmbedding, REGISTRY, build}``,
``encoders.{BaseTower, MeanPoolingTower, AveragePoolingTower, TwoTower, TOWER_REGISTRY,
build_tower, build_two_tower}``, ``losses.{contrastive_triplet_loss, multiple_negatives_loss,
in_batch_sampled_softmax_loss, LOSS_REGISTRY, build}``; plus ``optim.AdamW`` (fused table
update), ``distributed`` (RCCL data parallelism) and ``install()`` which registers these
classes into an importable reference ``twotower`` package so its train.py runs them unchanged.
"""
from __future__ import annotations

import importlib
import sys

from . import checkpoint, data, distributed, embeddings, encoders, losses, ops, optim, search
from .embeddings import BaseEmbedding, LookupEmbedding
from .encoders import (AveragePoolingTower, BaseTower, MeanPoolingTower, TOWER_REGISTRY, TwoTower, build_tower,
                       build_two_tower)
from .losses import (LOSS_REGISTRY, contrastive_triplet_loss, in_batch_sampled_softmax_loss,
                     multiple_negatives_loss)
from .train_step import TrainStep

__all__ = [
    "BaseEmbedding", "LookupEmbedding", "BaseTower", "MeanPoolingTower", "AveragePoolingTower", "TwoTower",
    "TOWER_REGISTRY", "LOSS_REGISTRY", "build_tower", "build_two_tower", "contrastive_triplet_loss",
    "multiple_negatives_loss", "in_batch_sampled_softmax_loss", "TrainStep", "install", "data", "distributed",
    "embeddings", "encoders", "losses", "ops", "optim", "checkpoint", "search",
]


def install(package: str = "twotower") -> None:
    """Point the reference package's registries/builders at the HIP implementations.

    Call before ``import twotower.train`` (its ``from .encoders import build_two_tower`` binds
    the name at import); names already bound in an imported ``twotower.train`` are patched too.
    """
    emb = importlib.import_module(f"{package}.embeddings")
    enc = importlib.import_module(f"{package}.encoders")
    los = importlib.import_module(f"{package}.losses")
    emb.REGISTRY["lookup"] = LookupEmbedding
    enc.TOWER_REGISTRY["mean"] = MeanPoolingTower
    enc.TOWER_REGISTRY["avg_pool"] = AveragePoolingTower
    enc.TwoTower = TwoTower
    enc.build_two_tower = build_two_tower
    for name, fn in LOSS_REGISTRY.items():
        los.LOSS_REGISTRY[name] = fn
    train_mod = sys.modules.get(f"{package}.train")
    if train_mod is not None:
        train_mod.build_two_tower = build_two_tower
