"""Micro-benchmark of the fused in-batch scorer (fwd + bwd) at bench shapes; prints us and TFLOP/s."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from twotower_amd import ops, _lib

def run(B, M, H, dt, iters=20):
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.nn.functional.normalize(torch.randn(B, H, device="cuda", generator=g), dim=-1).requires_grad_(True)
    d = torch.nn.functional.normalize(torch.randn(M, H, device="cuda", generator=g), dim=-1).requires_grad_(True)
    for _ in range(3):
        ops.in_batch_softmax_loss(q, d, 0.1, compute_dtype=dt).backward()
    torch.cuda.synchronize()
    _lib.TIMER.reset(); _lib.TIMER.enabled = True
    for _ in range(iters):
        ops.in_batch_softmax_loss(q, d, 0.1, compute_dtype=dt).backward()
    _lib.TIMER.enabled = False
    s = _lib.TIMER.summary()
    f, b = s["tt_inbatch_fwd"]["mean_ms"], s["tt_inbatch_bwd"]["mean_ms"]
    mult = 2 if dt == "bf16_split" else 1  # hi/lo split doubles the second product
    ex_f = (2 + 2 * mult) * B * M * H; ex_b = ex_f
    return dict(B=B, M=M, H=H, dt=dt, fwd_us=round(f * 1e3, 1), bwd_us=round(b * 1e3, 1),
                algo_tflops=round(6 * B * M * H / ((f + b) * 1e-3) / 1e12, 1),
                executed_tflops=round((ex_f + ex_b) / ((f + b) * 1e-3) / 1e12, 1))

cases = [(8192, 16384, 256, "bf16"), (8192, 16384, 256, "bf16_split"), (8192, 8192, 256, "bf16"),
         (4096, 8192, 128, "fp32"), (4096, 8192, 128, "bf16")]
for c in cases:
    print(json.dumps(run(*c)), flush=True)
