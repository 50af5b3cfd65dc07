"""Diagnostic (not a test; run with TT_INBATCH_BWD=stored): the forward's stored P of a cold
first call against a second call on the same inputs, block by block."""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from twotower_amd import _lib  # noqa: E402

DEV = "cuda"
L = _lib.lib()
B, M, H = 300, 700, 64
g = torch.Generator(device=DEV).manual_seed(1)
q = torch.nn.functional.normalize(torch.randn(B, H, device=DEV, generator=g), dim=-1)
d = torch.nn.functional.normalize(torch.randn(M, H, device=DEV, generator=g), dim=-1)
nb = L.tt_inbatch_ws_size(B, M, H, _lib.TT_BF16)
al = lambda x: (x + 255) // 256 * 256  # noqa: E731
p_off = al((B + 64) * H * 2) + al((M + 64) * H * 2) + al((B + 64) * H * 2)
nqt, nct = (B + 127) // 128 * 4, (M + 127) // 128 * 4
Ps, dds = [], []
for call in range(3):
    ws = torch.zeros(nb + 512, dtype=torch.uint8, device=DEV)
    base = (ws.data_ptr() + 255) // 256 * 256 - ws.data_ptr()
    lse, rows, loss = torch.empty(B, device=DEV), torch.empty(B, device=DEV), torch.empty((), device=DEV)
    dqu, dq, dd = torch.empty(B, H, device=DEV), torch.empty(B, H, device=DEV), torch.empty(M, H, device=DEV)
    st = torch.cuda.current_stream().cuda_stream
    _lib.call("tt_inbatch_fwd", q.data_ptr(), d.data_ptr(), B, M, H, _lib.TT_BF16, 10.0, 0, 1, lse.data_ptr(),
              rows.data_ptr(), loss.data_ptr(), dqu.data_ptr(), ws.data_ptr(), ws.numel(), st)
    torch.cuda.synchronize()
    Ps.append(ws[base + p_off: base + p_off + nqt * nct * 2048].clone().view(nct, nqt, 2048))
    gl = torch.tensor([1.0], device=DEV)
    _lib.call("tt_inbatch_bwd", q.data_ptr(), d.data_ptr(), B, M, H, _lib.TT_BF16, 10.0, 0, lse.data_ptr(),
              dqu.data_ptr(), gl.data_ptr(), 1.0 / B, dq.data_ptr(), dd.data_ptr(), ws.data_ptr(), ws.numel(), st)
    torch.cuda.synchronize()
    dds.append(dd.clone())
for c in (1, 2):
    diff = (Ps[0][:22] != Ps[c][:22]).any(-1).nonzero().tolist()
    print("P call0 vs call%d differing (ct, qt) blocks:" % c, diff[:20], len(diff), flush=True)
    bad = ((dds[0] - dds[c]).abs() > 1e-6).any(1).nonzero().flatten().tolist()
    print("dd rows differing call0 vs call%d:" % c, bad[:10], len(bad), flush=True)
print("zero P blocks call0:", (Ps[0][:22] == 0).all(-1).nonzero().tolist()[:20], flush=True)
