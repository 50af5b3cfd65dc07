"""Micro-benchmark: torch fp32 GEMM shapes of the tower head (N=3B rows, E=H=256)."""
import torch, time
dev = "cuda"
N, E, H = 24576, 256, 256
x = torch.randn(N, E, device=dev); W = torch.randn(H, E, device=dev); b = torch.randn(H, device=dev)
dy = torch.randn(N, H, device=dev)
def t(fn, n=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n): fn()
    e.record(); torch.cuda.synchronize(); return s.elapsed_time(e) / n * 1e3
res = {}
res["addmm fwd x@W^T+b"] = t(lambda: torch.addmm(b, x, W.t()))
res["mm dx = dy@W"] = t(lambda: dy @ W)
res["mm dW = dy^T@x"] = t(lambda: dy.t() @ x)
res["bmm splitK8 dW"] = t(lambda: torch.bmm(dy.view(8, N // 8, H).transpose(1, 2), x.view(8, N // 8, E)).sum(0))
res["db = dy.sum(0)"] = t(lambda: dy.sum(0))
for lib in ("hipblaslt", "rocblas"):
    try:
        torch.backends.cuda.preferred_blas_library(lib)
        res[f"[{lib}] addmm fwd"] = t(lambda: torch.addmm(b, x, W.t()))
        res[f"[{lib}] dW"] = t(lambda: dy.t() @ x)
        res[f"[{lib}] dx"] = t(lambda: dy @ W)
    except Exception as ex:
        res[f"[{lib}]"] = str(ex)
for k, v in res.items():
    print(f"{k:30s} {v if isinstance(v, str) else f'{v:8.1f} us'}")
