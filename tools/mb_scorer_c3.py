"""Scorer fwd/bwd device times at the C3 shape (B 8192, M 16384, H 256, bf16), HIP events per ABI call."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from twotower_amd import _lib, ops  # noqa: E402

B, M, H = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (8192, 16384, 256)))
g = torch.Generator(device="cuda").manual_seed(0)
q = torch.nn.functional.normalize(torch.randn(B, H, device="cuda", generator=g), dim=-1).requires_grad_(True)
d = torch.nn.functional.normalize(torch.randn(M, H, device="cuda", generator=g), dim=-1).requires_grad_(True)
for _ in range(3):
    ops.in_batch_softmax_loss(q, d, 0.1, compute_dtype="bf16").backward()
torch.cuda.synchronize()
_lib.TIMER.reset()
_lib.TIMER.enabled = True
for _ in range(20):
    ops.in_batch_softmax_loss(q, d, 0.1, compute_dtype="bf16").backward()
_lib.TIMER.enabled = False
s = _lib.TIMER.summary()
print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), "B": B, "M": M, "H": H,
                  "fwd_us": round(s["tt_inbatch_fwd"]["mean_ms"] * 1e3, 1),
                  "bwd_us": round(s["tt_inbatch_bwd"]["mean_ms"] * 1e3, 1)}))
