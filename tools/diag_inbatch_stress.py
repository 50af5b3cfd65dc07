"""Diagnostic (not a test): repeat the opt-in stored-probability bf16 backward (run with
TT_INBATCH_BWD=stored) on many inputs; each input twice, to tell a race (the two results differ)
from a data-dependent error (both wrong alike)."""
import os
import sys

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import reference_math as O  # noqa: E402
from twotower_amd import ops  # noqa: E402

DEV = "cuda"


def unit(rng, n, h):
    x = rng.standard_normal((n, h)).astype(np.float32)
    return x / np.linalg.norm(x, axis=1, keepdims=True)


bad = 0
for it in range(12):
    for (B, M, off, H) in [(300, 700, 0, 64), (300, 700, 0, 32), (129, 129, 0, 64), (300, 700, 0, 256)]:
        rng = np.random.default_rng(1000 * it + H)
        q = torch.as_tensor(unit(rng, B, H)).bfloat16().float()
        d = torch.as_tensor(unit(rng, M, H)).bfloat16().float()
        outs = []
        for rep in range(2):
            Q = q.to(DEV).requires_grad_(True)
            D = d.to(DEV).requires_grad_(True)
            ops.InBatchSoftmaxLoss.apply(Q, D, 10.0, off, "bf16", None).backward()
            outs.append(D.grad.double().cpu().numpy())
        _, (_, rdd), _ = O.in_batch_fwd_bwd(q.double().numpy(), d.double().numpy(), 0.1, g=1.0, label_off=off)
        errs = [float(np.nan_to_num(np.abs(o - rdd).max(), nan=1e9) / np.abs(rdd).max()) for o in outs]
        same = bool(np.array_equal(outs[0], outs[1], equal_nan=True))
        if max(errs) > 2e-3 or not same:
            bad += 1
            rows = np.nonzero(np.abs(outs[0] - rdd).max(1) > 1e-3 * np.abs(rdd).max())[0]
            print("BAD", it, (B, M, off, H), errs, "same", same, "rows", rows[:10].tolist(), len(rows), flush=True)
print("done, bad", bad, flush=True)
