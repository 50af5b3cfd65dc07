"""Diagnostic (not a test; TT_INBATCH_BWD=stored): the first bf16 in-batch call of a fresh process,
with or without a host sync between forward and backward (argv[1] == "sync")."""
import os
import sys

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import reference_math as O  # noqa: E402
from twotower_amd import ops  # noqa: E402

sync = len(sys.argv) > 1 and sys.argv[1] == "sync"
B, M, H = 300, 700, 64
rng = np.random.default_rng(64)
q = rng.standard_normal((B, H)).astype(np.float32)
d = rng.standard_normal((M, H)).astype(np.float32)
q = torch.as_tensor(q / np.linalg.norm(q, axis=1, keepdims=True)).bfloat16().float()
d = torch.as_tensor(d / np.linalg.norm(d, axis=1, keepdims=True)).bfloat16().float()
Q, D = q.cuda().requires_grad_(True), d.cuda().requires_grad_(True)
loss = ops.InBatchSoftmaxLoss.apply(Q, D, 10.0, 0, "bf16", None)
if sync:
    torch.cuda.synchronize()
loss.backward()
_, (_, rdd), _ = O.in_batch_fwd_bwd(q.double().numpy(), d.double().numpy(), 0.1, g=1.0, label_off=0)
err = float(np.nan_to_num(np.abs(D.grad.double().cpu().numpy() - rdd).max(), nan=1e9) / np.abs(rdd).max())
print("sync" if sync else "nosync", "err", err, "BAD" if err > 2e-3 else "ok", flush=True)
