"""Per-rank GPU cost of the two data-parallel table exchanges at N ranks, on one GPU (C3/C4 table:
V 200k, E 256, 3 x 8192 sequences of L 64 per rank), graph-replayed:
  gather: the fused scatter + AdamW over all N ranks' sequences (every rank runs it; the ids and
          d_pooled of the N ranks are what the all-gathers deliver);
  shard:  the dense table gradient of this rank's sequences (bag_mean_backward_planned over V x E)
          + AdamW on this rank's V/N rows (the collectives themselves are not timed here).
Link bytes per rank per step are printed for both (ring collectives: (N-1)/N of the gathered or
reduced size).  Usage: python tools/mb_table_sync.py [--ranks 1 2 4 8]"""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import twotower_amd as tt  # noqa: E402
from twotower_amd import _lib, ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ranks", type=int, nargs="*", default=[1, 2, 4, 8])
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()
B, L, V, E = 8192, 64, 200_000, 256
g = torch.Generator(device="cuda").manual_seed(0)
table = torch.randn(V, E, device="cuda", generator=g) * 0.02
m = torch.zeros_like(table)
v = torch.zeros_like(table)
args = torch.zeros(_lib.TT_ADAM_ARGS_BYTES // 4, device="cuda")
step = torch.zeros(1, device="cuda")
slot = _lib.AdamSlot(step.data_ptr(), args.data_ptr())
_lib.call("tt_adam_prepare", ctypes.byref(slot), 1, 1e-3, 0.9, 0.999, 1e-8, 0.01,
          torch.cuda.current_stream().cuda_stream)


def timed(fn, iters):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(iters):
            fn()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        gr.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (3 * iters) * 1e3


def batch_ids(seed):
    q, p, n = tt.data.synthetic_triplets(B, L, V, seed=seed, device="cuda")
    return torch.cat([q, p, n]).to(torch.int32).contiguous()


own = batch_ids(0)
for R in a.ranks:
    ids = torch.cat([own] + [batch_ids(1000 * r) for r in range(1, R)]).contiguous()
    N = ids.shape[0]
    d_pooled = torch.randn(N, E, device="cuda", generator=g)
    denom = (ids > 0).sum(1).float() + 1e-9
    plan = ops.BagPlan(ids, V, E, 0)
    plan.wait()
    t_gather = timed(lambda: ops.bag_mean_backward_adamw_planned(d_pooled, denom, plan, table, m, v, args), a.iters)
    # shard: this rank's dense gradient + AdamW on V/R rows
    nown = own.shape[0]
    plan1 = ops.BagPlan(own, V, E, 0)
    plan1.wait()
    gbuf = torch.empty(V, E, device="cuda")
    Vs = -(-V // R)
    t_scatter = timed(lambda: ops.bag_mean_backward_planned(d_pooled[:nown], denom[:nown], plan1, out=gbuf), a.iters)
    t_adam = timed(lambda: _lib.call("tt_adamw", table.data_ptr(), gbuf.data_ptr(), m.data_ptr(), v.data_ptr(), Vs * E,
                                     1e-3, 0.9, 0.999, 1e-8, 0.01, 1, torch.cuda.current_stream().cuda_stream), a.iters)
    link_gather = (R - 1) * nown * (L * 4 + E * 4 + 4)  # ids + d_pooled + denom of the other ranks
    link_shard = 2 * (R - 1) / R * V * E * 4               # reduce-scatter + all-gather of the table
    print(f"N={R}: gather-mode update {t_gather:.0f} us | shard-mode scatter {t_scatter:.0f} us + AdamW(V/N) "
          f"{t_adam:.0f} us | link MB per rank: gather {link_gather / 1e6:.0f}, shard {link_shard / 1e6:.0f}",
          flush=True)
    del d_pooled, plan, plan1, gbuf
    torch.cuda.empty_cache()
