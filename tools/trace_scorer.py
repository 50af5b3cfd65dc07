"""Region timeline of the bf16 scorer engine (forward, C3 shape) from a TT_SCORER_TRACE build:
per stage t, s_memtime at: stage start | vmcnt done | barrier done | after unit 0 | after unit 1.
Build: tools/build_variants.sh trace=-DTT_SCORER_TRACE (debug only); run: trace_scorer.py LIB."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from twotower_amd import ops, _lib
if len(sys.argv) > 1:  # a variant library built with -DTT_SCORER_TRACE (tools/build_variants.sh)
    _lib.LIB_PATH = os.path.abspath(sys.argv[1])

B, M, H = 8192, 16384, 256
g = torch.Generator(device="cuda").manual_seed(0)
q = torch.nn.functional.normalize(torch.randn(B, H, device="cuda", generator=g), dim=-1)
d = torch.nn.functional.normalize(torch.randn(M, H, device="cuda", generator=g), dim=-1)
for _ in range(3):
    ops.in_batch_softmax_loss(q, d, 0.1, compute_dtype="bf16")
torch.cuda.synchronize()
buf = (ctypes.c_longlong * 512)()
fn = _lib.lib().tt_debug_scorer_trace
fn.argtypes, fn.restype = [ctypes.c_void_p], ctypes.c_int
rc = fn(buf)
a = np.array(buf, dtype=np.int64).reshape(64, 8)
# slots (unit-stream forward): 0 stage start | 1 vmcnt done | 2 barrier done | 3 after unit 0 | 4 after unit 1
names = ["vmcnt", "barrier", "unit 0 (32 MFMA)", "unit 1 (32 MFMA)", "to next stage"]
rows = []
for t in range(1, 60):
    s = a[t]
    nxt = a[t + 1][0]
    rows.append([s[1] - s[0], s[2] - s[1], s[3] - s[2], s[4] - s[3], nxt - s[4], nxt - s[0]])
r = np.array(rows)
print("rc", rc)
print("cycles per stage region (median over stages 1..59):")
for n, v in zip(names + ["stage total"], np.median(r, 0)):
    print(f"  {n:18s} {v:8.0f}")
print("mean stage total", r[:, -1].mean(), " MFMA floor per stage 64*32 = 2048")
