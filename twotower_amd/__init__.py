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
    ``train.build_pipeline`` (train.py:298-371) is wrapped, now or when train is imported, so a
    config may opt in to the fused table update for the loop's own torch.optim.AdamW under a
    namespace the reference ignores: ``hip: {table_update: backward}`` (optim.fuse_table_update;
    default / ``optimizer``: the dense table gradient stepped by the optimizer, as before), and
    ``hip: {dense_update: backward}`` for the tower parameters (optim.fuse_dense_update: one
    multi-tensor AdamW launch at the end of backward instead of torch's foreach step).
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
        _patch_train(train_mod)
    elif not any(isinstance(f, _TrainImportHook) and f.name == f"{package}.train" for f in sys.meta_path):
        sys.meta_path.insert(0, _TrainImportHook(f"{package}.train"))


TABLE_UPDATES = ("optimizer", "backward")


def _patch_train(train_mod) -> None:
    train_mod.build_two_tower = build_two_tower
    orig = getattr(train_mod, "build_pipeline", None)
    if orig is None or getattr(orig, "_tt_wrapped", False):
        return

    def build_pipeline(config, device):
        hip = config.get("hip", {}) or {}
        mode = hip.get("table_update", "optimizer")
        dense = hip.get("dense_update", "optimizer")
        for key, val in (("table_update", mode), ("dense_update", dense)):
            if val not in TABLE_UPDATES:
                raise ValueError(f"hip.{key} must be one of {TABLE_UPDATES}, got {val!r}")
        model, dataset, optimizer, loss_fn = orig(config, device)
        if mode == "backward":
            optim.fuse_table_update(optimizer, model)
        if dense == "backward":
            optim.fuse_dense_update(optimizer, model)
        return model, dataset, optimizer, loss_fn

    build_pipeline._tt_wrapped = True
    build_pipeline.__wrapped__ = orig
    build_pipeline.__doc__ = orig.__doc__
    train_mod.build_pipeline = build_pipeline


class _TrainImportHook:
    """Patches ``<package>.train`` right after it is first imported (install() ran before it)."""

    def __init__(self, name: str):
        self.name = name

    def find_spec(self, fullname, path=None, target=None):
        if fullname != self.name:
            return None
        import importlib.machinery
        import importlib.util

        sys.meta_path.remove(self)
        try:
            spec = importlib.util.find_spec(fullname)
        finally:
            sys.meta_path.insert(0, self)
        if spec is None or spec.loader is None:
            return spec
        loader = spec.loader
        exec_module = loader.exec_module

        def exec_and_patch(module):
            exec_module(module)
            _patch_train(module)

        loader.exec_module = exec_and_patch
        return spec
