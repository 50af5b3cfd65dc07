"""Bag backward outputs (dense planned grad and the fused scatter + AdamW) on seeded uniform and
Zipf ids, saved for a bit-for-bit comparison between two library builds (TT_LIB).
Usage: plan_ab.py OUT.pt"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from twotower_amd import ops, _lib
DEV = "cuda"
out = {}
for name, V, E, nseq, L, zipf in (("uniform", 200_000, 256, 24576, 64, None), ("zipf", 50_000, 256, 6000, 64, 1.05),
                                  ("small", 997, 64, 203, 12, None), ("hot", 3000, 128, 4000, 64, 1.3)):
    rng = np.random.default_rng(7)
    if zipf:
        ids = np.minimum(rng.zipf(zipf, size=(nseq, L)), V - 1)
    else:
        ids = rng.integers(1, V, size=(nseq, L))
    ids[:, L // 2:] *= (rng.random((nseq, L - L // 2)) > 0.3)
    ids = torch.as_tensor(ids, device=DEV, dtype=torch.int32)
    dp = torch.as_tensor(rng.standard_normal((nseq, E)).astype(np.float32), device=DEV)
    den = torch.clamp((ids > 0).sum(1).float(), min=1.0)
    g = ops.bag_mean_backward(dp, den, ids, V, 0, _lib.TT_SCATTER_SORTED)
    plan = ops.BagPlan(ids, V, E, 0)
    g2 = ops.bag_mean_backward_planned(dp, den, plan)
    torch.cuda.synchronize()
    out[name] = (g.cpu(), g2.cpu())
torch.save(out, sys.argv[1])
print("saved", sys.argv[1])
