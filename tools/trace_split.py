"""Region timelines of the split-bf16 fp32 engines (score_split_fwd_kernel, score_split_ddp_kernel;
C2 shape) from a TT_SCORER_TRACE build (debug only: tools/build_variants.sh trace=-DTT_SCORER_TRACE).
Per unit t of workgroup 0, wave 0: s_memtime at region boundaries and s_memrealtime at unit start
(the in-kernel clock); per workgroup s_memrealtime at entry / loop start / loop end / exit.
Usage: trace_split.py LIB [B M H]."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from twotower_amd import _lib, ops  # noqa: E402

_lib.LIB_PATH = os.path.abspath(sys.argv[1])
B, M, H = (int(x) for x in sys.argv[2:5]) if len(sys.argv) >= 5 else (4096, 8192, 128)
g = torch.Generator(device="cuda").manual_seed(0)
q = torch.nn.functional.normalize(torch.randn(B, H, device="cuda", generator=g), dim=-1).requires_grad_(True)
d = torch.nn.functional.normalize(torch.randn(M, H, device="cuda", generator=g), dim=-1).requires_grad_(True)
for _ in range(200):  # >= 2 s of back-to-back launches would be the clock rule; this is the steady state of a step loop
    ops.in_batch_softmax_loss(q, d, 0.1, compute_dtype="fp32").backward()
torch.cuda.synchronize()
buf = (ctypes.c_longlong * 512)()
fn = _lib.lib().tt_debug_scorer_trace
fn.argtypes, fn.restype = [ctypes.c_void_p], ctypes.c_int
fn(buf)
a = np.array(buf, dtype=np.int64).reshape(64, 8)
n = int((a[:, 0] > 0).sum())
rows = []
for t in range(1, n - 1):
    s = a[t]
    rows.append([s[1] - s[0], s[3] - s[1], a[t + 1][0] - s[3], a[t + 1][0] - s[0]])
r = np.array(rows)
print(f"forward units traced {n}")
for name, v in zip(["start -> barrier point (14 steps, 84 MFMA)", "vmcnt wait + barrier", "barrier -> next unit (2 steps, 12 MFMA)",
                    "unit total"], np.median(r, 0)):
    print(f"  {name:44s} {v:8.0f} cyc")
clk = (a[n - 2][0] - a[1][0]) / ((a[n - 2][2] - a[1][2]) / 100e6) / 1e9
print(f"  in-kernel clock {clk:.2f} GHz; MFMA floor per unit 96 x 32 = 3072 cyc")

buf = (ctypes.c_longlong * 512)()
fn = _lib.lib().tt_debug_scorer_trace_bwd
fn.argtypes, fn.restype = [ctypes.c_void_p], ctypes.c_int
fn(buf)
a = np.array(buf, dtype=np.int64).reshape(64, 8)
n = int((a[:, 0] > 0).sum())
rows = [[a[t][1] - a[t][0], a[t][2] - a[t][1], a[t][3] - a[t][2], a[t + 1][0] - a[t][3], a[t + 1][0] - a[t][0]]
        for t in range(1, n - 1)]
r = np.array(rows)
print(f"backward units traced {n}")
for name, v in zip(["start: P(t+1) wait", "-> barrier point (6 steps, 36 MFMA)", "vmcnt wait + barrier",
                    "barrier -> next unit (2 steps, 12 MFMA)", "unit total"], np.median(r, 0)):
    print(f"  {name:44s} {v:8.0f} cyc")
clk = (a[n - 2][0] - a[1][0]) / ((a[n - 2][4] - a[1][4]) / 100e6) / 1e9
print(f"  in-kernel clock {clk:.2f} GHz; MFMA floor per unit 48 x 32 = 1536 cyc")

kb = (ctypes.c_longlong * 8192)()
fk = _lib.lib().tt_debug_scorer_ktrace
fk.argtypes, fk.restype = [ctypes.c_void_p], ctypes.c_int
fk(kb)
for which, base in (("forward (score_split_fwd_kernel)", 4096), ("backward (score_split_ddp_kernel)", 0)):
    k = np.array(kb[base:base + 4096], dtype=np.int64).reshape(1024, 4)
    k = k[k[:, 0] > 0]
    t0 = k[:, 0].min()
    us = (k - t0) / 100.0
    print(f"{which}: workgroups traced {len(k)}")
    for name, col in (("entry", 0), ("loop start", 1), ("loop end", 2), ("exit", 3)):
        c = us[:, col]
        print(f"  {name:10s} min {c.min():7.2f} med {np.median(c):7.2f} max {c.max():7.2f} us")
    print(f"  prologue med {np.median(us[:, 1] - us[:, 0]):.2f} us; loop med {np.median(us[:, 2] - us[:, 1]):.2f} "
          f"(min {np.min(us[:, 2] - us[:, 1]):.2f} max {np.max(us[:, 2] - us[:, 1]):.2f}); epilogue med "
          f"{np.median(us[:, 3] - us[:, 2]):.2f} us")
