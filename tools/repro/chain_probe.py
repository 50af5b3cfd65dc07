"""Diagnostics for the fused head chains (head_chain.hip) and the tt_head_gemm shapes the chains and
LinearHead use: prints, per case, the max relative error against float64 and, for the chain's second
product with W2 = I and b2 = 0 (so y must equal h), where h's values land in y.
Usage: python tools/repro/chain_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from twotower_amd import _lib, ops  # noqa: E402

DEV = "cuda"


def rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))


g = torch.Generator(device=DEV).manual_seed(0)
# 1. tt_head_gemm epi 4 / epi 0 / epi 3 on every (K, N) against float64
for K, N in ((256, 256), (128, 128), (64, 128), (256, 128), (128, 256), (64, 256), (128, 64), (256, 64)):
    x = torch.randn(1000, K, device=DEV, generator=g)
    W = torch.randn(N, K, device=DEV, generator=g) / K ** 0.5
    b = torch.randn(N, device=DEV, generator=g)
    ref = x.double() @ W.double().T
    res = {}
    for epi in (4, 0, 3):
        if (epi in (4, 0) and N == 64) or (epi == 3 and False):
            continue
        try:
            mask = torch.empty(_lib.lib().tt_head_relu_mask_bytes(1000) // 4, dtype=torch.int32, device=DEV)
            y = ops._head_gemm(x, ops._planes(W, False), epi, bias=b, mask=mask, N=N)
            want = {4: ref + b.double(), 0: torch.relu(ref + b.double()), 3: ref}[epi]
            res[epi] = f"{rel(y, want):.2e}"
        except Exception as e:  # noqa: BLE001
            res[epi] = f"refused ({str(e)[:60]})"
    print(f"tt_head_gemm K {K} N {N}: {res}", flush=True)
# 2. the chain's second product with W2 = I, b2 = 0: y must equal h
for E, H in ((256, 256), (128, 128), (64, 128)):
    rows = 256
    x = torch.randn(rows, E, device=DEV, generator=g)
    W1 = torch.randn(H, E, device=DEV, generator=g) / E ** 0.5
    b1 = torch.zeros(H, device=DEV) + 0.5
    W2 = torch.eye(H, device=DEV)
    b2 = torch.zeros(H, device=DEV)
    p1, p2 = ops._planes(W1, False), ops._planes(W2, False)
    bits = torch.empty(_lib.lib().tt_head_chain_bits_bytes(rows, H) // 4, dtype=torch.int32, device=DEV)
    h, y = torch.empty(rows, H, device=DEV), torch.empty(rows, H, device=DEV)
    ops.call("tt_head_fwd_chain", x.data_ptr(), rows, E, E, H, p1.data_ptr(), p2.data_ptr(), b1.data_ptr(),
             b2.data_ptr(), bits.data_ptr(), h.data_ptr(), y.data_ptr(), None, 0, _lib.stream_of(x))
    torch.cuda.synchronize()
    print(f"chain E {E} H {H}: h vs float64 {rel(h, torch.relu(x.double() @ W1.double().T + 0.5)):.2e}, "
          f"y vs h {rel(y, h):.2e}", flush=True)
    hc, yc = h.cpu(), y.cpu()
    for r, c in ((0, 0), (0, 1), (0, 4), (0, 8), (0, 16), (1, 0), (4, 0), (0, 32), (0, 100)):
        v = yc[r, c].item()
        hits = (hc == v).nonzero().tolist()[:3]
        print(f"   y[{r},{c}] = {v:.6f} found in h at {hits}", flush=True)
print("done", flush=True)
