"""Standalone time of the fused table update (tt_bag_mean_bwd_adamw_planned: scale rows + per-row
reduce + AdamW) at the bench shape (C3: V 200k, E 256, 3 x 8192 sequences of L 64), graph-replayed.
The plan is built once; the per-step AdamW scalars are prepared once (the timing does not depend
on their values).  Usage: python tools/mb_bag_bwd.py [--zipf S] [--iters N]"""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import twotower_amd as tt  # noqa: E402
from twotower_amd import _lib, ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--zipf", type=float, default=None)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
B, L, V, E = 8192, 64, 200_000, 256
q, p, n = tt.data.synthetic_triplets(B, L, V, seed=0, device="cuda", zipf_s=a.zipf)
ids = torch.cat([q, p, n]).to(torch.int32).contiguous()
N = ids.shape[0]
g = torch.Generator(device="cuda").manual_seed(0)
table = torch.randn(V, E, device="cuda", generator=g) * 0.02
m = torch.zeros_like(table)
v = torch.zeros_like(table)
d_pooled = torch.randn(N, E, device="cuda", generator=g)
denom = (ids > 0).sum(1).float() + 1e-9
plan = ops.BagPlan(ids, V, E, 0)
plan.wait()
step = torch.zeros(1, device="cuda")
args = torch.zeros(_lib.TT_ADAM_ARGS_BYTES // 4, device="cuda")


slot = _lib.AdamSlot(step.data_ptr(), args.data_ptr())
_lib.call("tt_adam_prepare", ctypes.byref(slot), 1, 1e-3, 0.9, 0.999, 1e-8, 0.01,
          torch.cuda.current_stream().cuda_stream)


def apply():
    ops.bag_mean_backward_adamw_planned(d_pooled, denom, plan, table, m, v, args)


s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        apply()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr):
    for _ in range(a.iters):
        apply()
gr.replay()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 5
e0.record()
for _ in range(reps):
    gr.replay()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / (a.iters * reps) * 1e3
algo = N * E * 4 + N * 4 + 24 * V * E
nnz = int((ids > 0).sum())
print(f"bag bwd+AdamW apply ({os.environ.get('TT_BAG_REDUCE', 'default')}, zipf={a.zipf}): {us:.1f} us  "
      f"algorithmic {algo / us / 1e3:.0f} GB/s  (+ gathered gs rows {(algo + nnz * E * 4) / us / 1e3:.0f} GB/s)")

# ---- reference points on the same buffers: dense AdamW over V x E (reads p, g, m, v; writes
# p, m, v = 28 B/param) and a plain device copy of one table
if os.environ.get("MB_REFS", "1") == "1":
    grad = torch.randn(V, E, device="cuda", generator=g)

    def dense():
        _lib.call("tt_adamw", table.data_ptr(), grad.data_ptr(), m.data_ptr(), v.data_ptr(), V * E, 1e-3, 0.9,
                  0.999, 1e-8, 0.01, 1, torch.cuda.current_stream().cuda_stream)

    dst = torch.empty_like(table)

    def copy():
        dst.copy_(table)

    for name, fn, nbytes in (("dense AdamW", dense, 28 * V * E), ("copy", copy, 8 * V * E)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(f"{name} over V x E: {us:.1f} us  {nbytes / us / 1e3:.0f} GB/s")

# ---- the dense-gradient apply (data parallel 'shard' mode writes the V x E gradient)
if os.environ.get("MB_DENSE", "1") == "1":
    gout = torch.empty(V, E, device="cuda")

    def dense_apply():
        ops.bag_mean_backward_planned(d_pooled, denom, plan, out=gout)

    for _ in range(3):
        dense_apply()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(20):
        dense_apply()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    print(f"bag bwd dense-grad apply ({os.environ.get('TT_BAG_REDUCE', 'default')}): {us:.1f} us  "
          f"{(N * E * 4 + N * 4 + V * E * 4) / us / 1e3:.0f} GB/s algorithmic")
