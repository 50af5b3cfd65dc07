"""Checkpoints in the reference's format (twotower/utils.py:231-330): one torch.save'd dict with
'model' (model.state_dict()), 'vocab' (tokeniser string_to_index), 'epoch', 'loss', 'timestamp'
and optionally 'optimizer' (optimizer.state_dict()).

Parameter names match the reference's modules (tests/golden/state_dict.npz pins them), so a
checkpoint written here loads with the reference's load_checkpoint into its TwoTower and vice
versa.  Tensors are saved on the CPU; a row-sharded table optimizer (data parallel, "shard" sync)
contributes its full-size moments (AdamW.state_dict gathers them), so the optimizer state also
loads into torch.optim.AdamW.  Loading uses torch.load(weights_only=True): nothing in the file is
executed.
"""
from __future__ import annotations

import datetime
import logging
import os
from typing import Any

import torch

logger = logging.getLogger("twotower_amd.checkpoint")


def _to_cpu(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj


def save_checkpoint(model: torch.nn.Module, tokeniser_vocab: dict[str, int],
                    optimizer: torch.optim.Optimizer | None = None, epoch: int = 0, loss: float = float("inf"),
                    checkpoint_dir: str = "checkpoints", checkpoint_name: str | None = None,
                    save_best: bool = True) -> str:
    """Same arguments, file name scheme and dict keys as the reference (utils.py:231-296)."""
    os.makedirs(checkpoint_dir, exist_ok=True)
    timestamp = datetime.datetime.now().strftime("%Y%m%d_%H%M%S")
    if checkpoint_name is None:
        checkpoint_name = f"two_tower_{timestamp}_epoch{epoch}.pt"
    path = os.path.join(checkpoint_dir, checkpoint_name)
    ckpt: dict[str, Any] = {"model": _to_cpu(model.state_dict()), "vocab": tokeniser_vocab, "epoch": epoch,
                            "loss": loss, "timestamp": timestamp}
    if optimizer is not None:
        ckpt["optimizer"] = _to_cpu(optimizer.state_dict())
    if torch.distributed.is_available() and torch.distributed.is_initialized() and torch.distributed.get_rank() != 0:
        return path  # every rank holds the same replicated state; rank 0 writes
    torch.save(ckpt, path)
    logger.info(f"Saved checkpoint to {path}")
    if save_best:
        torch.save(ckpt, os.path.join(checkpoint_dir, "best_model.pt"))
    return path


def load_checkpoint(checkpoint_path: str, model: torch.nn.Module | None = None,
                    optimizer: torch.optim.Optimizer | None = None, device: str = "cpu") -> dict[str, Any]:
    """Same behaviour as the reference (utils.py:298-330), with the safe loader."""
    ckpt = torch.load(checkpoint_path, map_location=device, weights_only=True)
    logger.info(f"Loaded checkpoint from {checkpoint_path} (epoch {ckpt.get('epoch', 'unknown')}, "
                f"loss {ckpt.get('loss', 'unknown')})")
    if model is not None and "model" in ckpt:
        model.load_state_dict(ckpt["model"])
    if optimizer is not None and "optimizer" in ckpt:
        optimizer.load_state_dict(ckpt["optimizer"])
    return ckpt
