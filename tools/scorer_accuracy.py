"""Error of each scorer compute dtype against the float64 oracle on fp32 inputs (what the bf16
modes cost end to end, input rounding included), and their kernel times.
    python tools/scorer_accuracy.py [B M H]"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import twotower_amd as tt  # noqa: E402
from oracle import reference_math as O  # noqa: E402

B, M, H = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (2048, 4096, 256)
rng = np.random.default_rng(0)
q = rng.standard_normal((B, H))
q /= np.linalg.norm(q, axis=1, keepdims=True)
d = rng.standard_normal((M, H))
d /= np.linalg.norm(d, axis=1, keepdims=True)
d[:B] = 0.7 * q + 0.3 * d[:B]  # positives correlated with their queries
d /= np.linalg.norm(d, axis=1, keepdims=True)
rl, (rdq, rdd), _ = O.in_batch_fwd_bwd(q, d, 0.1)


def rel(a, b):
    return float(np.abs(a - b).max() / np.abs(b).max())


for dt in ("fp32", "bf16_split", "bf16"):
    qt = torch.tensor(q, dtype=torch.float32, device="cuda", requires_grad=True)
    dtt = torch.tensor(d, dtype=torch.float32, device="cuda", requires_grad=True)
    loss = tt.ops.in_batch_softmax_loss(qt, dtt, 0.1, compute_dtype=dt)
    loss.backward()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    for _ in range(3):
        ev[0].record()
        l2 = tt.ops.in_batch_softmax_loss(qt, dtt, 0.1, compute_dtype=dt)
        ev[1].record()
        l2.backward()
        ev[2].record()
    torch.cuda.synchronize()
    print(f"{dt:10s} loss rel {abs(loss.item() - rl) / rl:.2e}  dq rel {rel(qt.grad.cpu().numpy() / 4, rdq):.2e}  "
          f"dd rel {rel(dtt.grad.cpu().numpy() / 4, rdd):.2e}  fwd {ev[0].elapsed_time(ev[1]):.3f} ms  "
          f"bwd {ev[1].elapsed_time(ev[2]):.3f} ms")
