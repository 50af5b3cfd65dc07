"""Debug: fused head-normalise + scorer prep vs unfused, per-buffer differences."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
import twotower_amd as tt
from twotower_amd import ops, _lib
from twotower_amd._lib import call, ptr

DEV = "cuda"
torch.manual_seed(0)
B, M, H = 300, 600, 256
rows = B + M
dt = _lib.compute_dtype_code("bf16")
W = torch.randn(H, H, device=DEV) * 0.05
b = torch.randn(H, device=DEV) * 0.1
h = torch.randn(rows, H, device=DEV)
planes = ops._planes(W, False)
na = torch.empty(rows, device=DEV); nb_ = torch.empty(rows, device=DEV)
ya = ops._head_gemm(h, planes, 1, bias=b, norms=na)
yb = ops._head_gemm(h, planes, 4, bias=b)
nbytes = _lib.lib().tt_inbatch_ws_size(B, M, H, dt)
wsa = torch.zeros(nbytes, dtype=torch.uint8, device=DEV)
wsb = torch.zeros(nbytes, dtype=torch.uint8, device=DEV)
call("tt_inbatch_l2_prep", ptr(yb), B, M, H, dt, ptr(nb_), ptr(wsb), nbytes, ops.stream_of(yb))
outs = []
for y, ws, entry in ((ya, wsa, "tt_inbatch_fwd"), (yb, wsb, "tt_inbatch_fwd_prepped")):
    lse = torch.empty(B, device=DEV); r = torch.empty(B, device=DEV); loss = torch.empty((), device=DEV)
    dqu = torch.empty(B, H, device=DEV)
    call(entry, ptr(y), ptr(y[B:]), B, M, H, dt, 10.0, 0, 1, ptr(lse), ptr(r), ptr(loss), ptr(dqu), ptr(ws), nbytes, ops.stream_of(y))
    g = torch.ones(1, device=DEV); dq = torch.empty(B, H, device=DEV); dd = torch.empty(M, H, device=DEV)
    call("tt_inbatch_bwd", ptr(y), ptr(y[B:]), B, M, H, dt, 10.0, 0, ptr(lse), ptr(dqu), ptr(g), 1.0 / B, ptr(dq), ptr(dd), ptr(ws), nbytes, ops.stream_of(y))
    outs.append((lse, r, loss, dqu, dq, dd))
torch.cuda.synchronize()
print("y equal", torch.equal(ya, yb), "norms equal", torch.equal(na, nb_), (na - nb_).abs().max().item())
for name, a, c in zip(("lse", "rows", "loss", "dqu", "dq", "dd"), outs[0], outs[1]):
    print(name, torch.equal(a, c), (a - c).abs().max().item())
diff = (wsa != wsb).nonzero()
print("ws bytes differ:", diff.numel(), diff[:10].flatten().tolist(), diff[-10:].flatten().tolist() if diff.numel() else [])
