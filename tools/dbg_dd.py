import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from twotower_amd import ops
from oracle import reference_math as O
for (B, M, H) in [(300, 700, 64), (300, 640, 64), (256, 700, 64), (320, 700, 64), (300, 768, 64)]:
    rng = np.random.default_rng(1)
    q = rng.standard_normal((B, H)); q /= np.linalg.norm(q, axis=1, keepdims=True)
    d = rng.standard_normal((M, H)); d /= np.linalg.norm(d, axis=1, keepdims=True)
    q = torch.tensor(q, dtype=torch.float32).bfloat16().float(); d = torch.tensor(d, dtype=torch.float32).bfloat16().float()
    Q = q.cuda().requires_grad_(True); D = d.cuda().requires_grad_(True)
    ops.InBatchSoftmaxLoss.apply(Q, D, 10.0, 0, "bf16", None).backward()
    _, (rdq, rdd), _ = O.in_batch_fwd_bwd(q.double().numpy(), d.double().numpy(), 0.1)
    err = np.abs(D.grad.double().cpu().numpy() - rdd).max(1) / np.abs(rdd).max()
    bad = np.nonzero(err > 1e-3)[0]
    print(B, M, H, "bad rows:", len(bad), bad[:10], bad[-5:] if len(bad) else "")
