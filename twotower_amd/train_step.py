"""One training step of the two-tower model, the body of the reference's hot loop
(twotower/train.py:103-139: forward :120-122, loss :133, zero_grad/backward/step :137-139),
with optional data parallelism.  Returns the loss as a device tensor (no host sync; the
reference's per-step .item() monitors at :144-154 are left to the caller).
"""
from __future__ import annotations

import torch

from .distributed import GradSync, is_active


class TrainStep:
    def __init__(self, model: torch.nn.Module, loss_fn, optimizer: torch.optim.Optimizer, group=None):
        self.model = model
        self.loss_fn = loss_fn
        self.optimizer = optimizer
        self.group = group
        self.sync = GradSync(model.parameters(), group=group) if is_active(group) else None

    def __call__(self, queries: torch.Tensor, positive_docs: torch.Tensor, negative_docs: torch.Tensor) -> torch.Tensor:
        q, p, n = self.model(queries, positive_docs, negative_docs)
        loss = self.loss_fn(q, p, n)
        self.optimizer.zero_grad(set_to_none=True)
        if self.sync is not None:
            (loss * self.sync.loss_scale()).backward()
            self.sync.sync()
        else:
            loss.backward()
        self.optimizer.step()
        return loss.detach()
