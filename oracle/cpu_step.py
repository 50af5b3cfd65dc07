"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): the CPU baseline.

A torch-on-CPU restatement of the reference's training step exactly as the reference computes
it (twotower/train.py:120-139 driving embeddings.py:30,40, encoders.py:62-77, losses.py,
torch.optim.AdamW): nn.Embedding gather -> mask multiply -> sum / (count + 1e-9) ->
Linear-ReLU-Linear -> F.normalize, the loss, dense backward, dense AdamW.  bench.py times it on
the GPU box's host cores as `cpu_baseline` (kind "port"); the reference source never travels.
"""
from __future__ import annotations

import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class RefTower(nn.Module):
    def __init__(self, V: int, E: int, H: int):
        super().__init__()
        self.embedding = nn.Embedding(V, E, padding_idx=0)              # embeddings.py:30
        self.feed_forward = nn.Sequential(nn.Linear(E, H), nn.ReLU(), nn.Linear(H, H))  # encoders.py:38-42

    def forward(self, ids):
        mask = (ids > 0).float().unsqueeze(-1)                           # encoders.py:62
        emb = self.embedding(ids) * mask                                 # :67
        pooled = emb.sum(1) / (mask.sum(1) + 1e-9)                       # :72
        return F.normalize(self.feed_forward(pooled), dim=-1)            # :77


def ref_loss(name: str, q, p, n, temperature=0.1, margin=0.2):
    if name == "triplet":                                                # losses.py:9-44
        return F.relu(margin - F.cosine_similarity(q, p, dim=1) + F.cosine_similarity(q, n, dim=1)).mean()
    if name == "in_batch":                                               # losses.py:88-118 on cat[p, n] (or p)
        d = p if n is None else torch.cat([p, n])
        logits = (q @ d.T) / temperature
        return F.cross_entropy(logits, torch.arange(q.shape[0], device=q.device))
    if name == "multiple_negatives":                                     # losses.py:47-85, n (B*K, H)
        d = torch.cat([p.unsqueeze(1), n.view(q.shape[0], -1, q.shape[1])], dim=1)
        logits = F.cosine_similarity(q.unsqueeze(1).expand_as(d), d, dim=2) / temperature
        return F.cross_entropy(logits, torch.zeros(q.shape[0], dtype=torch.long))
    raise ValueError(name)


def host_cores() -> dict:
    """Physical cores this process may run on (affinity mask x /proc/cpuinfo core ids), the logical
    CPUs in the mask, and the threads torch will use."""
    import os

    cpus = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    phys, cur = {}, {}
    try:
        for line in open("/proc/cpuinfo"):
            if ":" not in line:
                if "processor" in cur:
                    phys[int(cur["processor"])] = (cur.get("physical id", "0"), cur.get("core id", cur["processor"]))
                cur = {}
                continue
            k, v = (x.strip() for x in line.split(":", 1))
            cur[k] = v
        if "processor" in cur:
            phys[int(cur["processor"])] = (cur.get("physical id", "0"), cur.get("core id", cur["processor"]))
    except OSError:
        pass
    cores = len({phys.get(c, ("?", c)) for c in cpus})
    return {"physical_cores": cores, "logical_cpus": len(cpus), "torch_threads": torch.get_num_threads()}


def time_cpu_step(V: int, E: int, H: int, batches, loss: str = "in_batch", threads: int | None = None,
                  min_seconds: float = 10.0, max_steps: int = 20) -> dict:
    """Pairs/s of the reference CPU step on `batches` (list of (q, p, n) int64 CPU tensors): the
    body of train_epoch (twotower/train.py:103-166) without its tqdm bar and W&B calls.  Runs at
    least 2 and at most max_steps steps, stopping once min_seconds have passed."""
    if threads:
        torch.set_num_threads(threads)
    torch.manual_seed(0)
    tower = RefTower(V, E, H)
    opt = torch.optim.AdamW(tower.parameters(), lr=1e-3)

    def step(b):
        q, p = b[0], b[1]
        n = b[2] if len(b) > 2 else None                                 # (q, p) pairs: no negatives
        qv, pv = tower(q), tower(p)                                      # tied towers (char_tower.yml)
        nv = tower(n) if n is not None else None
        loss_v = ref_loss(loss, qv, pv, nv)
        opt.zero_grad()
        loss_v.backward()
        opt.step()
        with torch.no_grad():  # the loop's per-batch monitors (train.py:143-156)
            F.cosine_similarity(qv, pv).mean().item()
            if nv is not None:
                F.cosine_similarity(qv, nv[:qv.shape[0]]).mean().item()
        loss_v.item()
        return loss_v

    step(batches[0])                                                     # warm-up
    t0 = time.perf_counter()
    steps, pairs = 0, 0
    while steps < max_steps and (time.perf_counter() - t0 < min_seconds or steps < 2):
        b = batches[steps % len(batches)]
        step(b)
        steps += 1
        pairs += b[0].shape[0]
    dt = time.perf_counter() - t0
    return {"pairs_per_s": pairs / dt, "steps": steps, "seconds": dt, "threads": torch.get_num_threads()}
