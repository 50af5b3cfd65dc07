"""Head GEMM kernels vs hipBLASLt at the bench shape (24576 x 256 x 256)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from twotower_amd import ops

N = 24576
x = torch.randn(N, 256, device="cuda")
W = torch.randn(256, 256, device="cuda") / 16
b = torch.randn(256, device="cuda")
P = ops._planes(W, False)
norms = torch.empty(N, device="cuda")


def t(fn, it=20, reps=10):
    """Per-call time from HIP graph replay of `it` back-to-back calls (no host launch overhead)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(it):
            fn()
    for _ in range(3):
        g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (it * reps) * 1e3


mask = torch.empty(N, 8, dtype=torch.int32, device="cuda")
ops._head_gemm(x, P, 0, bias=b, mask=mask)
for epi in range(4):
    us = t(lambda: ops._head_gemm(x, P, epi, bias=b, mask=mask, norms=norms))
    print(f"head_gemm epi {epi}: {us:.1f} us  ({2 * N * 256 * 256 / us / 1e6:.1f} TFLOP/s fp32-equivalent)")
print(f"split planes: {t(lambda: ops._planes(W, True)):.1f} us")
print(f"torch addmm: {t(lambda: torch.addmm(b, x, W.t())):.1f} us")
print(f"torch addmm+relu: {t(lambda: torch._addmm_activation(b, x, W.t())):.1f} us")
g2 = torch.randn(N, 256, device="cuda")
print(f"head_wgrad (dW + db): {t(lambda: ops.head_wgrad(g2, x)):.1f} us")
print(f"K-split library wgrad + colsum: {t(lambda: (ops._weight_grad(g2, x), ops.colsum(g2))):.1f} us")
