"""Per-rank GPU cost of the data-parallel table exchanges at N ranks, measured on one GPU (the
collectives themselves need the 8-GPU node; their link bytes per rank are printed).  Graph-replayed.

Configs: c3 (the C3/C4 table: V 200k, E 256, 3 x 8192 sequences of L 64 per rank) and c5
(configs[4]: V 1M, E 256, 8192 queries x (1 positive + 4 negatives) = 6 x 8192 sequences per rank).

  gather: every rank runs the fused scatter + AdamW over all N ranks' sequences (the ids and
          d_pooled / denom of the N ranks are what the all-gathers deliver);
  shard:  the dense table gradient of this rank's sequences (V x E) + AdamW on this rank's V/N rows;
          links: reduce-scatter of the gradient + all-gather of the updated rows;
  owner:  every rank's ids and d_pooled / denom all-gathered (as gather), but each rank scatters and
          updates only the rows it owns (V/N: moments sharded as in shard), then the updated rows are
          all-gathered: emulated here by remapping the N ranks' ids to this rank's rows (others ->
          padding) and running the fused update over a V/N-row table, plus the sort plan over all
          N ranks' ids (the plan the owner needs).
Usage: python tools/mb_table_sync.py [--config c3|c5] [--ranks 1 2 4 8]"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import twotower_amd as tt  # noqa: E402
from twotower_amd import _lib, ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3", choices=["c3", "c5"])
ap.add_argument("--ranks", type=int, nargs="*", default=[1, 2, 4, 8])
ap.add_argument("--iters", type=int, default=5)
a = ap.parse_args()
B, L, E = 8192, 64, 256
V, K = (200_000, 1) if a.config == "c3" else (1_000_000, 4)
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
    q, p, n = tt.data.synthetic_triplets(B, L, V, seed=seed, device="cuda", negatives=K)
    return torch.cat([q, p, n]).to(torch.int32).contiguous()


own = batch_ids(0)
nown = own.shape[0]
for R in a.ranks:
    ids = torch.cat([own] + [batch_ids(1000 * r) for r in range(1, R)]).contiguous()
    N = ids.shape[0]
    d_pooled = torch.randn(N, E, device="cuda", generator=g)
    denom = (ids > 0).sum(1).float() + 1e-9
    res = {"config": a.config, "ranks": R, "tokens_per_rank": int((own > 0).sum())}
    # gather: plan over all ranks' ids + the replicated fused update
    t_plan_all = timed(lambda: ops.BagPlan(ids, V, E, 0).wait(), a.iters)
    plan = ops.BagPlan(ids, V, E, 0)
    plan.wait()
    res["gather_update_us"] = timed(
        lambda: ops.bag_mean_backward_adamw_planned(d_pooled, denom, plan, table, m, v, args), a.iters)
    res["plan_all_ranks_us"] = t_plan_all
    del plan
    # shard: this rank's dense gradient + AdamW on V/R rows
    plan1 = ops.BagPlan(own, V, E, 0)
    plan1.wait()
    gbuf = torch.empty(V, E, device="cuda")
    Vs = -(-V // R)
    res["plan_own_us"] = timed(lambda: ops.BagPlan(own, V, E, 0).wait(), a.iters)
    res["shard_dense_grad_us"] = timed(
        lambda: ops.bag_mean_backward_planned(d_pooled[:nown], denom[:nown], plan1, out=gbuf), a.iters)
    res["shard_adamw_us"] = timed(
        lambda: _lib.call("tt_adamw", table.data_ptr(), gbuf.data_ptr(), m.data_ptr(), v.data_ptr(), Vs * E, 1e-3, 0.9,
                          0.999, 1e-8, 0.01, 1, torch.cuda.current_stream().cuda_stream), a.iters)
    del plan1, gbuf
    # owner: the N ranks' ids remapped to this rank's Vs rows (rank 0 owns rows [0, Vs)), others padding
    own_ids = torch.where(ids < Vs, ids, torch.zeros_like(ids)).contiguous()
    res["owner_plan_us"] = timed(lambda: ops.BagPlan(own_ids, Vs, E, 0).wait(), a.iters)
    plan_o = ops.BagPlan(own_ids, Vs, E, 0)
    plan_o.wait()
    res["owner_update_us"] = timed(
        lambda: ops.bag_mean_backward_adamw_planned(d_pooled, denom, plan_o, table[:Vs], m[:Vs], v[:Vs], args),
        a.iters)
    del plan_o, own_ids
    row_b = E * 4
    seq_b = L * 4 + E * 4 + 4  # ids + d_pooled + denom per sequence
    res["link_MB_per_rank"] = {
        "gather": (R - 1) * nown * seq_b / 1e6,
        "shard": 2 * (R - 1) / R * V * row_b / 1e6,
        "owner": ((R - 1) * nown * seq_b + (R - 1) / R * V * row_b) / 1e6,
    }
    res = {k: (round(x, 1) if isinstance(x, float) else x) for k, x in res.items()}
    res["link_MB_per_rank"] = {k: round(x, 1) for k, x in res["link_MB_per_rank"].items()}
    print(json.dumps(res), flush=True)
    del d_pooled, ids, denom
    torch.cuda.empty_cache()
