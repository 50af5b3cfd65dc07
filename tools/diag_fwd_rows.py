"""Diagnostic (not a test): per-row forward lse of the bf16 scorer vs float64 on the rounded operands;
prints which query rows are wrong and how (pattern by row % 128, per-candidate-count)."""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from twotower_amd import _lib  # noqa: E402

if len(sys.argv) > 1:
    _lib.LIB_PATH = os.path.abspath(sys.argv[1])
DEV = "cuda"
L = _lib.lib()
for (B, M, H) in [(64, 64, 256), (64, 128, 256), (64, 192, 256), (128, 256, 256), (300, 700, 256), (64, 64, 32)]:
    g = torch.Generator(device=DEV).manual_seed(1)
    q = torch.nn.functional.normalize(torch.randn(B, H, device=DEV, generator=g), dim=-1)
    d = torch.nn.functional.normalize(torch.randn(M, H, device=DEV, generator=g), dim=-1)
    nb = L.tt_inbatch_ws_size(B, M, H, _lib.TT_BF16)
    ws = torch.zeros((nb // 4 + 64,), device=DEV)
    lse, rows = torch.empty(B, device=DEV), torch.empty(B, device=DEV)
    loss = torch.empty((), device=DEV)
    dqu = torch.empty(B, H, device=DEV)
    st = torch.cuda.current_stream().cuda_stream
    _lib.call("tt_inbatch_fwd", q.data_ptr(), d.data_ptr(), B, M, H, _lib.TT_BF16, 10.0, 0, 1, lse.data_ptr(),
              rows.data_ptr(), loss.data_ptr(), dqu.data_ptr(), ws.data_ptr(), ws.numel() * 4, st)
    torch.cuda.synchronize()
    qb, db = q.bfloat16().double(), d.bfloat16().double()
    ref = torch.logsumexp(qb @ db.T * 10.0, 1)
    err = (lse.double() - ref).abs()
    bad = (err > 1e-3) | ~torch.isfinite(lse)
    idx = bad.nonzero().flatten().tolist()
    print((B, M, H), "bad rows", len(idx), "first", idx[:12], "lse sample", lse[:4].tolist(), "ref", ref[:4].tolist(),
          flush=True)
