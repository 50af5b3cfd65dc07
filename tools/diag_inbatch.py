"""Diagnostic (not a test): bf16 in-batch fwd + bwd through the C ABI with a NaN-filled workspace,
to find reads of workspace bytes the forward did not write."""
import os
import sys

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402
import torch  # noqa: E402

from twotower_amd import _lib  # noqa: E402

DEV = "cuda"
L = _lib.lib()
for (B, M, off, H) in [(300, 700, 0, 64), (300, 700, 0, 256), (129, 129, 0, 64), (300, 700, 0, 32), (300, 700, 0, 128)]:
    g = torch.Generator(device=DEV).manual_seed(1)
    q = torch.nn.functional.normalize(torch.randn(B, H, device=DEV, generator=g), dim=-1)
    d = torch.nn.functional.normalize(torch.randn(M, H, device=DEV, generator=g), dim=-1)
    nb = L.tt_inbatch_ws_size(B, M, H, _lib.TT_BF16)
    res = []
    for fill in (0.0, float("nan")):
        ws = torch.full((nb // 4 + 64,), fill, device=DEV)
        lse, rows = torch.empty(B, device=DEV), torch.empty(B, device=DEV)
        loss = torch.empty((), device=DEV)
        dqu, dq, dd = torch.empty(B, H, device=DEV), torch.empty(B, H, device=DEV), torch.empty(M, H, device=DEV)
        gl = torch.tensor([1.0], device=DEV)
        st = torch.cuda.current_stream().cuda_stream
        _lib.call("tt_inbatch_fwd", q.data_ptr(), d.data_ptr(), B, M, H, _lib.TT_BF16, 10.0, off, 1, lse.data_ptr(),
                  rows.data_ptr(), loss.data_ptr(), dqu.data_ptr(), ws.data_ptr(), ws.numel() * 4, st)
        _lib.call("tt_inbatch_bwd", q.data_ptr(), d.data_ptr(), B, M, H, _lib.TT_BF16, 10.0, off, lse.data_ptr(),
                  dqu.data_ptr(), gl.data_ptr(), 1.0 / B, dq.data_ptr(), dd.data_ptr(), ws.data_ptr(), ws.numel() * 4, st)
        torch.cuda.synchronize()
        nanrows = torch.isnan(dd).any(1).nonzero().flatten().tolist()
        res.append((fill, float(loss), bool(torch.isnan(dq).any()), len(nanrows), nanrows[:8]))
        if fill == 0.0:
            dd0 = dd.clone()
    print((B, M, off, H), res, "max|dd0-dd|", float((dd0 - dd).abs().nan_to_num(1e9).max()), flush=True)
