"""Region timeline of the stored-probability scorer backward (score_ddp_kernel, C3 shape) from a
TT_SCORER_TRACE build: per stage t, s_memtime at: stage start | tile 0 done | vmcnt done | barrier
done | stage end.  Build: tools/build_variants.sh trace=-DTT_SCORER_TRACE; run: trace_scorer_bwd.py LIB."""
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
buf = (ctypes.c_longlong * 512)()
fn = _lib.lib().tt_debug_scorer_trace_bwd
fn.argtypes, fn.restype = [ctypes.c_void_p], ctypes.c_int
rc = fn(buf)
a = np.array(buf, dtype=np.int64).reshape(64, 8)
names = ["tile 0 (16 MFMA)", "vmcnt", "barrier", "tile 1 (16 MFMA)", "to next stage"]
rows = []
for t in range(1, 30):
    s = a[t]
    rows.append([s[1] - s[0], s[2] - s[1], s[3] - s[2], s[4] - s[3], a[t + 1][0] - s[4], a[t + 1][0] - s[0]])
r = np.array(rows)
print("rc", rc)
for n, v in zip(names + ["stage total"], np.median(r, 0)):
    print(f"  {n:18s} {v:8.0f}")
print("MFMA floor per stage 32*32 = 1024")

# kernel-level: per workgroup (wave 0) s_memrealtime (100 MHz) at entry / loop start / loop end / exit
kb = (ctypes.c_longlong * 8192)()
fk = _lib.lib().tt_debug_scorer_ktrace
fk.argtypes, fk.restype = [ctypes.c_void_p], ctypes.c_int
fk(kb)
for which, base in (("backward (score_ddp_kernel)", 0), ("forward (score_bf16_kernel)", 4096)):
    k = np.array(kb[base:base + 4096], dtype=np.int64).reshape(1024, 4)
    k = k[k[:, 0] > 0]
    if not len(k):
        continue
    t0 = k[:, 0].min()
    us = (k - t0) / 100.0  # 100 MHz ticks -> us
    print(f"{which}: workgroups traced {len(k)}")
    for name, col in (("entry", 0), ("loop start", 1), ("loop end", 2), ("exit", 3)):
        c = us[:, col]
        print(f"  {name:10s} min {c.min():7.2f} med {np.median(c):7.2f} max {c.max():7.2f} us")
    print(f"  prologue (entry->loop) med {np.median(us[:, 1] - us[:, 0]):.2f} us; loop med {np.median(us[:, 2] - us[:, 1]):.2f}"
          f" (min {np.min(us[:, 2] - us[:, 1]):.2f} max {np.max(us[:, 2] - us[:, 1]):.2f}); epilogue med "
          f"{np.median(us[:, 3] - us[:, 2]):.2f} us")
