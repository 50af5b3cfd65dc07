"""Stage timeline of the folded forward combine (FwdFold) from a TT_SCORER_TRACE build, C3 shape:
per workgroup s_memrealtime (100 MHz) at fold entry | publish drained | ticket taken | partials
folded | rows done | (last block) mean ticket | mean done, and the engine's loop start / end.
Build: tools/build_variants.sh trace=-DTT_SCORER_TRACE; run: trace_fold.py tools/variants/lib_trace.so"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from twotower_amd import _lib, ops  # noqa: E402

if len(sys.argv) > 1:
    _lib.LIB_PATH = os.path.abspath(sys.argv[1])
B, M, H = 8192, 16384, 256
g = torch.Generator(device="cuda").manual_seed(0)
q = torch.nn.functional.normalize(torch.randn(B, H, device="cuda", generator=g), dim=-1).requires_grad_(True)
d = torch.nn.functional.normalize(torch.randn(M, H, device="cuda", generator=g), dim=-1).requires_grad_(True)
for _ in range(3):
    ops.in_batch_softmax_loss(q, d, 0.1, compute_dtype="bf16").backward()
torch.cuda.synchronize()
kb = (ctypes.c_longlong * 8192)()
fk = _lib.lib().tt_debug_scorer_ktrace
fk.argtypes, fk.restype = [ctypes.c_void_p], ctypes.c_int
fk(kb)
fb = (ctypes.c_longlong * 8192)()
ff = _lib.lib().tt_debug_scorer_ftrace
ff.argtypes, ff.restype = [ctypes.c_void_p], ctypes.c_int
ff(fb)
k = np.array(kb[4096:8192], dtype=np.int64).reshape(1024, 4)
f = np.array(fb[:], dtype=np.int64).reshape(1024, 8)
n = int((k[:, 0] > 0).sum())
k, f = k[:n], f[:n]
t0 = k[:, 0].min()
us = lambda x: (x - t0) / 100.0  # noqa: E731
print(f"workgroups {n}")
for name, col in (("entry", 0), ("loop start", 1), ("loop end", 2)):
    c = us(k[:, col])
    print(f"  {name:12s} min {c.min():7.2f} med {np.median(c):7.2f} max {c.max():7.2f}")
names = ["fold entry", "published", "ticket", "folded", "rows done", "mean ticket", "mean done"]
for col, name in enumerate(names):
    v = f[:, col]
    v = v[v > 0]
    if len(v) == 0:
        continue
    c = us(v)
    print(f"  {name:12s} n {len(v):4d} min {c.min():7.2f} med {np.median(c):7.2f} max {c.max():7.2f}")
