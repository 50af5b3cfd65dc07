"""Region timeline of the bf16 scorer engine (forward, C3 shape) from a TT_SCORER_TRACE build:
per stage t, s_memtime at: jt0 start | jt0 S+map end | jt1 start | drain done | barrier done |
jt1 S+map end.  Build: make -C twotower_amd/csrc EXTRA=-DTT_SCORER_TRACE (debug only)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from twotower_amd import ops, _lib

B, M, H = 8192, 16384, 256
g = torch.Generator(device="cuda").manual_seed(0)
q = torch.nn.functional.normalize(torch.randn(B, H, device="cuda", generator=g), dim=-1)
d = torch.nn.functional.normalize(torch.randn(M, H, device="cuda", generator=g), dim=-1)
for _ in range(3):
    ops.in_batch_softmax_loss(q, d, 0.1, compute_dtype="bf16")
torch.cuda.synchronize()
buf = (ctypes.c_longlong * 512)()
rc = _lib.lib().tt_debug_scorer_trace(buf)
a = np.array(buf, dtype=np.int64).reshape(64, 8)
names = ["jt0 S+map", "jt0 acc", "jt1 drain", "jt1 barrier", "jt1 S+map", "jt1 acc(next)"]
# slots: 0 jt0 start, 3 jt0 before acc, 4 jt1 start, 5 drain done, 6 barrier done, 7 jt1 before acc
rows = []
for t in range(1, 60):
    s = a[t]
    nxt = a[t + 1][0]
    rows.append([s[3] - s[0], s[4] - s[3], s[5] - s[4], s[6] - s[5], s[7] - s[6], nxt - s[7], nxt - s[0]])
r = np.array(rows)
print("rc", rc)
print("cycles per stage region (median over stages 1..59):")
for n, v in zip(names + ["stage total"], np.median(r, 0)):
    print(f"  {n:14s} {v:8.0f}")
print("mean stage total", r[:, -1].mean(), " MFMA floor per stage 64*32 = 2048")
