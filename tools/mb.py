"""Microbenchmarks of the step's kernels on one GPU, one driver with a subcommand per op family
(device times from HIP graph replay of back-to-back calls, or HIP events per C-ABI call).

  python tools/mb.py bag_bwd [c3|c5] [--zipf S]  fused table update (scale rows + per-row reduce +
                                                 AdamW) at C3, against a dense AdamW, a device copy and
                                                 the dense-gradient apply on the same buffers
  python tools/mb.py plan [c3|c5]                the backward's sort plan (tt_bag_plan), uniform and Zipf
  python tools/mb.py head                        the tower head GEMMs (24576 x 256 x 256) against hipBLASLt
  python tools/mb.py scorer [B M H dtype ...]    in-batch scorer fwd / bwd (prep + engine + combine)
  python tools/mb.py scorer_dp [dtype]           one rank's scorer passes at the N-rank shapes (N = 1..8,
                                                 cross-device negatives, candidate-owner gradients)
  python tools/mb.py split_fwd                   two-launch vs one-launch data-parallel forward
  python tools/mb.py table_sync [c3|c5]          per-rank GPU cost of the table exchanges at N ranks
                                                 (gather / shard / owner) and their link bytes
  python tools/mb.py column_sync [c5|c3]         per-rank GPU cost and link bytes of the column-sharded table
                                                 (table_sync "column") at N = 1, 2, 4, 8
  python tools/mb.py l2prep                      the head's normalise fused with the scorer's operand prep,
                                                 alone (C3 and B x B rows)
  python tools/mb.py scorer_once B M H [dtype] [lib]   three scorer fwd + bwd calls, nothing else (for
                                                 counter collection: tools/pmc_scorer.sh)
  python tools/mb.py next_rows                   SURVEY section 8(f) rows: the device feeder's batch gather,
                                                 forward-only encode, cosine scores + top-k over a 1M-document
                                                 index, and the AveragePoolingTower head (LinearHead +
                                                 LayerNorm/L2), each against its HBM roofline and a torch form
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import twotower_amd as tt  # noqa: E402
from twotower_amd import _lib, ops  # noqa: E402
from twotower_amd._lib import call, ptr  # noqa: E402

DEV = "cuda"


def graph_us(fn, iters: int = 10, reps: int = 5) -> float:
    """Per-call device time of `fn` from the replay of a graph holding `iters` back-to-back calls."""
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
    for _ in range(reps):
        gr.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (iters * reps) * 1e3


def event_us(fn, iters: int = 20) -> float:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def adam_args():
    step = torch.zeros(1, device=DEV)
    args = torch.zeros(_lib.TT_ADAM_ARGS_BYTES // 4, device=DEV)
    slot = _lib.AdamSlot(step.data_ptr(), args.data_ptr())
    call("tt_adam_prepare", ctypes.byref(slot), 1, 1e-3, 0.9, 0.999, 1e-8, 0.01, torch.cuda.current_stream().cuda_stream)
    return step, args


def ids_for(B, L, V, K=1, seed=0, zipf=None):
    q, p, n = tt.data.synthetic_triplets(B, L, V, seed=seed, device=DEV, zipf_s=zipf, negatives=K)
    return torch.cat([q, p, n]).to(torch.int32).contiguous()


# ------------------------------------------------------------------------------------------------
def bag_bwd(a):
    B, L, E = 8192, 64, 256
    V, K = (1_000_000, 4) if a.shape == "c5" else (200_000, 1)  # C5: multi_pos_multi_neg, 1M rows
    ids = ids_for(B, L, V, K, zipf=a.zipf)
    N = ids.shape[0]
    g = torch.Generator(device=DEV).manual_seed(0)
    table = torch.randn(V, E, device=DEV, generator=g) * 0.02
    m, v = torch.zeros_like(table), torch.zeros_like(table)
    d_pooled = torch.randn(N, E, device=DEV, generator=g)
    denom = (ids > 0).sum(1).float() + 1e-9
    plan = ops.BagPlan(ids, V, E, 0)
    plan.wait()
    _, args = adam_args()
    us = graph_us(lambda: ops.bag_mean_backward_adamw_planned(d_pooled, denom, plan, table, m, v, args), 20)
    algo = N * E * 4 + N * 4 + 24 * V * E
    print(f"fused update ({a.shape or 'c3'}, zipf={a.zipf}): {us:.1f} us, algorithmic {algo / us / 1e3:.0f} GB/s")
    # where the gathers are served from: the same plan with every sorted sequence
    # index folded into the first K sequences, so the gathered gs rows fit an XCD's L2 (K = 4096: a
    # 1 MB slice per XCD) or the Infinity Cache, at the same row structure and counts.  Timing only
    # (the sums are of other rows): if the real plan runs as fast as the L2-resident one, the
    # gathers that miss L2 cost no HBM time.
    offs = (ctypes.c_int64 * 3)()
    call("tt_bag_plan_layout", plan.nseq, plan.L, plan.V, plan.E, offs)
    b0 = (-plan.buf.data_ptr()) % 256
    vals = plan.buf[b0 + offs[1]: b0 + offs[1] + 4 * plan.nseq * plan.L].view(torch.int32)
    keep = vals.clone()
    for K in (4096, 16384, N):
        vals.copy_(torch.remainder(keep, K))
        us_k = graph_us(lambda: ops.bag_mean_backward_adamw_planned(d_pooled, denom, plan, table, m, v, args), 20)
        print(f"fused update, gathers from the first {K} sequences ({K * E / 1e6:.1f} MB per XCD slice): "
              f"{us_k:.1f} us")
    vals.copy_(keep)
    grad = torch.randn(V, E, device=DEV, generator=g)
    dst = torch.empty_like(table)
    dense = lambda: call("tt_adamw", ptr(table), ptr(grad), ptr(m), ptr(v), V * E, 1e-3, 0.9, 0.999, 1e-8,  # noqa
                         0.01, 1, torch.cuda.current_stream().cuda_stream)
    for name, fn, nb in (("dense AdamW over V x E", dense, 28 * V * E), ("device copy of the table",
                                                                         lambda: dst.copy_(table), 8 * V * E)):
        us = event_us(fn)
        print(f"{name}: {us:.1f} us, {nb / us / 1e3:.0f} GB/s")
    us = event_us(lambda: ops.bag_mean_backward_planned(d_pooled, denom, plan, out=dst))
    print(f"dense-gradient apply: {us:.1f} us, {(N * E * 4 + N * 4 + V * E * 4) / us / 1e3:.0f} GB/s algorithmic")


def plan(a):
    shape = a.shape or "c3"
    B, L, E = 8192, 64, 256
    V, K = (1_000_000, 4) if shape == "c5" else (200_000, 1)
    for name, z in (("uniform", None), ("zipf1.0", 1.0)):
        ids = ids_for(B, L, V, K, zipf=z)
        print(f"tt_bag_plan {shape} {name}: {graph_us(lambda: ops.BagPlan(ids, V, E, 0).wait()):.1f} us")


def head(a):
    N = 24576
    x = torch.randn(N, 256, device=DEV)
    W = torch.randn(256, 256, device=DEV) / 16
    b = torch.randn(256, device=DEV)
    P = ops._planes(W, False)
    norms = torch.empty(N, device=DEV)
    mask = torch.empty(N, 8, dtype=torch.int32, device=DEV)
    for epi in range(4):
        us = graph_us(lambda: ops._head_gemm(x, P, epi, bias=b, mask=mask, norms=norms), 20)
        print(f"head_gemm epi {epi}: {us:.1f} us")
    g2 = torch.randn(N, 256, device=DEV)
    print(f"split planes: {graph_us(lambda: ops._planes(W, True), 20):.1f} us")
    print(f"torch addmm (hipBLASLt): {graph_us(lambda: torch.addmm(b, x, W.t()), 20):.1f} us")
    print(f"head_wgrad (dW + db): {graph_us(lambda: ops.head_wgrad(g2, x), 20):.1f} us")


def scorer(a):
    cases = [tuple(a.rest[i:i + 4]) for i in range(0, len(a.rest), 4)] or [
        (8192, 16384, 256, "bf16"), (8192, 8192, 256, "bf16"), (4096, 8192, 128, "fp32")]
    for B, M, H, dt in cases:
        B, M, H = int(B), int(M), int(H)
        g = torch.Generator(device=DEV).manual_seed(0)
        q = torch.nn.functional.normalize(torch.randn(B, H, device=DEV, generator=g), dim=-1).requires_grad_(True)
        d = torch.nn.functional.normalize(torch.randn(M, H, device=DEV, generator=g), dim=-1).requires_grad_(True)
        for _ in range(3):
            ops.in_batch_softmax_loss(q, d, 0.1, compute_dtype=dt).backward()
        torch.cuda.synchronize()
        _lib.TIMER.reset()
        _lib.TIMER.enabled = True
        for _ in range(20):
            ops.in_batch_softmax_loss(q, d, 0.1, compute_dtype=dt).backward()
        _lib.TIMER.enabled = False
        s = _lib.TIMER.summary()
        f, b = s["tt_inbatch_fwd"]["mean_ms"], s["tt_inbatch_bwd"]["mean_ms"]
        print(json.dumps(dict(B=B, M=M, H=H, dt=dt, fwd_us=round(f * 1e3, 1), bwd_us=round(b * 1e3, 1),
                              algo_tflops=round(6 * B * M * H / ((f + b) * 1e-3) / 1e12, 1))), flush=True)


def scorer_dp(a):
    B, H, T, P = 8192, 256, _lib.TT_INBATCH_TAIL_ROWS, _lib.TT_INBATCH_MAX_PARTS
    M = 2 * B
    dt = _lib.compute_dtype_code(a.shape or "bf16")
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device=DEV).manual_seed(0)
    unit = lambda n: torch.nn.functional.normalize(torch.randn(n, H, device=DEV, generator=g), dim=-1)  # noqa
    for W in (1, 2, 4, 8):
        q, d_all, q_all = unit(B), unit(W * M), unit(W * B)
        qb = torch.empty(B + T, H, dtype=torch.bfloat16, device=DEV)
        qn = torch.empty(B, device=DEV)
        call("tt_inbatch_prep_rows", ptr(q), B, H, ptr(qb), ptr(qn), None, st)
        db_all = torch.empty(W * M + T, H, dtype=torch.bfloat16, device=DEV)
        parts = torch.empty(P, device=DEV)
        call("tt_inbatch_prep_rows", ptr(d_all), W * M, H, ptr(db_all), None, ptr(parts), st)
        qb_all = torch.empty(W * B + T, H, dtype=torch.bfloat16, device=DEV)
        call("tt_inbatch_prep_rows", ptr(q_all), W * B, H, ptr(qb_all), None, None, st)
        db = db_all[:M + T]
        ws = torch.empty(_lib.lib().tt_inbatch_ex_ws_size(B, W * M, W * B, M, H, dt), dtype=torch.uint8, device=DEV)
        lse, lse2, rows = (torch.empty(B, device=DEV) for _ in range(3))
        loss = torch.empty((), device=DEV)
        dqu, dq, dd = torch.empty(B, H, device=DEV), torch.empty(B, H, device=DEV), torch.empty(M, H, device=DEV)
        lse2_all = torch.empty(W * B + T, device=DEV)
        gl = torch.ones(1, device=DEV)

        def fwd():
            call("tt_inbatch_fwd_ex", ptr(qb), ptr(qn), B, ptr(db_all), ptr(parts), P, W * M, H, dt, 10.0, 0, 1,
                 ptr(lse), ptr(lse2), ptr(rows), ptr(loss), ptr(dqu), ptr(ws), ws.numel(), st)

        fwd()
        lse2_all[:W * B] = lse2.repeat(W)
        lse2_all[W * B:] = float("inf")

        def bwd():
            call("tt_inbatch_bwd_ex", ptr(qb_all), ptr(lse2_all), W * B, 0, ptr(db), M, B, 0, H, dt, 10.0, ptr(dqu),
                 ptr(gl), 1.0 / B, ptr(dq), ptr(dd), ptr(ws), ws.numel(), st)

        tf, tb = event_us(fwd, 10), event_us(bwd, 10)
        fl = 4.0 * B * W * M * H
        print(json.dumps({"world": W, "candidates": W * M, "fwd_us": round(tf, 1), "bwd_us": round(tb, 1),
                          "fwd_tflops": round(fl / tf / 1e6, 1), "bwd_tflops": round(fl / tb / 1e6, 1)}), flush=True)


def split_fwd(a):
    B, M, H, T, P = 8192, 16384, 256, _lib.TT_INBATCH_TAIL_ROWS, _lib.TT_INBATCH_MAX_PARTS
    dt = _lib.compute_dtype_code("bf16")
    g = torch.Generator(device=DEV).manual_seed(0)
    st = torch.cuda.current_stream().cuda_stream
    for N in (2, 4, 8):
        rank = N // 2
        q = torch.nn.functional.normalize(torch.randn(B, H, device=DEV, generator=g), dim=-1)
        d_all = torch.nn.functional.normalize(torch.randn(N * M, H, device=DEV, generator=g), dim=-1)
        qb = torch.empty(B + T, H, dtype=torch.bfloat16, device=DEV)
        qn = torch.empty(B, device=DEV)
        call("tt_inbatch_prep_rows", ptr(q), B, H, ptr(qb), ptr(qn), None, st)
        db_all = torch.zeros(N * M + T, H, dtype=torch.bfloat16, device=DEV)
        parts_all = torch.zeros(N * P, device=DEV)
        for r in range(N):
            call("tt_inbatch_prep_rows", ptr(d_all[r * M:(r + 1) * M]), M, H, ptr(db_all[r * M:]), None,
                 ptr(parts_all[r * P:]), st)
        db = torch.zeros(M + T, H, dtype=torch.bfloat16, device=DEV)
        db[:M] = db_all[rank * M:(rank + 1) * M]
        parts = parts_all[rank * P:(rank + 1) * P].clone()
        ws = torch.empty(_lib.lib().tt_inbatch_ex_ws_size(B, N * M, N * B, M, H, dt), dtype=torch.uint8, device=DEV)
        lse, lse2, rows = (torch.empty(B, device=DEV) for _ in range(3))
        loss = torch.empty((), device=DEV)
        dqu = torch.empty(B, H, device=DEV)
        one = lambda: call("tt_inbatch_fwd_ex", ptr(qb), ptr(qn), B, ptr(db_all), ptr(parts_all), N * P, N * M,  # noqa
                           H, dt, 10.0, rank * M, 1, ptr(lse), ptr(lse2), ptr(rows), ptr(loss), ptr(dqu), ptr(ws),
                           ws.numel(), st)

        def two():
            call("tt_inbatch_fwd_ex_local", ptr(qb), ptr(qn), B, ptr(db), ptr(parts), P, M, N * M, rank * M, H, dt,
                 10.0, ptr(ws), ws.numel(), st)
            call("tt_inbatch_fwd_ex_remote", ptr(qb), ptr(qn), B, ptr(db_all), ptr(parts_all), N * P, ptr(parts), P,
                 M, N * M, rank * M, H, dt, 10.0, 1, ptr(lse), ptr(lse2), ptr(rows), ptr(loss), ptr(dqu), ptr(ws),
                 ws.numel(), st)

        t1, t2 = event_us(one, 10), event_us(two, 10)
        print(f"N={N}: one launch {t1:.1f} us, two launches {t2:.1f} us")


def table_sync(a):
    """gather: every rank runs the fused scatter + AdamW over all N ranks' sequences; shard: this
    rank's dense V x E gradient + AdamW on V/N rows (links: reduce-scatter + all-gather); owner: the
    N ranks' ids remapped to this rank's rows (others padding) and the fused update over a V/N-row
    table, plus the sort plan over all N ranks' ids (links: factored all-gather + row all-gather)."""
    B, L, E = 8192, 64, 256
    shape = a.shape or "c3"
    V, K = (200_000, 1) if shape == "c3" else (1_000_000, 4)
    g = torch.Generator(device=DEV).manual_seed(0)
    table = torch.randn(V, E, device=DEV, generator=g) * 0.02
    m, v = torch.zeros_like(table), torch.zeros_like(table)
    _, args = adam_args()
    own = ids_for(B, L, V, K, zipf=a.zipf)
    nown = own.shape[0]
    for R in (1, 2, 4, 8):
        ids = torch.cat([own] + [ids_for(B, L, V, K, seed=1000 * r, zipf=a.zipf) for r in range(1, R)]).contiguous()
        N = ids.shape[0]
        d_pooled = torch.randn(N, E, device=DEV, generator=g)
        denom = (ids > 0).sum(1).float() + 1e-9
        res = {"config": shape, "ranks": R, "tokens_per_rank": int((own > 0).sum())}
        res["plan_all_ranks_us"] = graph_us(lambda: ops.BagPlan(ids, V, E, 0).wait())
        pl = ops.BagPlan(ids, V, E, 0)
        pl.wait()
        res["gather_update_us"] = graph_us(lambda: ops.bag_mean_backward_adamw_planned(d_pooled, denom, pl, table, m,
                                                                                       v, args))
        del pl
        p1 = ops.BagPlan(own, V, E, 0)
        p1.wait()
        gbuf = torch.empty(V, E, device=DEV)
        Vs = -(-V // R)
        res["plan_own_us"] = graph_us(lambda: ops.BagPlan(own, V, E, 0).wait())
        res["shard_dense_grad_us"] = graph_us(lambda: ops.bag_mean_backward_planned(d_pooled[:nown], denom[:nown], p1,
                                                                                    out=gbuf))
        res["shard_adamw_us"] = graph_us(lambda: call("tt_adamw", ptr(table), ptr(gbuf), ptr(m), ptr(v), Vs * E, 1e-3,
                                                      0.9, 0.999, 1e-8, 0.01, 1,
                                                      torch.cuda.current_stream().cuda_stream))
        del p1, gbuf
        own_ids = torch.where(ids < Vs, ids, torch.zeros_like(ids)).contiguous()
        res["owner_plan_us"] = graph_us(lambda: ops.BagPlan(own_ids, Vs, E, 0).wait())
        po = ops.BagPlan(own_ids, Vs, E, 0)
        po.wait()
        res["owner_update_us"] = graph_us(lambda: ops.bag_mean_backward_adamw_planned(d_pooled, denom, po, table[:Vs],
                                                                                      m[:Vs], v[:Vs], args))
        del po, own_ids
        seq_b = L * 4 + E * 4 + 4  # ids + d_pooled + denom per sequence
        res = {k: (round(x, 1) if isinstance(x, float) and k != "zipf" else x) for k, x in res.items()}
        res["link_MB_per_rank"] = {"gather": round((R - 1) * nown * seq_b / 1e6, 1),
                                   "shard": round(2 * (R - 1) / R * V * E * 4 / 1e6, 1),
                                   "owner": round(((R - 1) * nown * seq_b + (R - 1) / R * V * E * 4) / 1e6, 1)}
        print(json.dumps(res), flush=True)
        del d_pooled, ids, denom
        torch.cuda.empty_cache()


def column_sync(a):
    """table_sync "column" at N ranks, per rank (the N ranks' sequences simulated by N independent
    batches on one GPU): the forward gather of this rank's E/N columns for every rank's sequences
    from its (V, E/N) slab, the two layout copies around the all-to-alls, the fused slab update from
    the N per-rank plans merged in the reduce (tt_bag_col_reduce), against the one-GPU gather and
    fused update of the rank's own batch (full width); plus the link bytes per rank: ids all-gather,
    pooled and gs all-to-alls (exposed) and the plan all-gather (issued on the plan's stream during
    the forward)."""
    B, L, E = 8192, 64, 256
    shape = a.shape or "c5"
    V, K = (200_000, 1) if shape == "c3" else (1_000_000, 4)
    g = torch.Generator(device=DEV).manual_seed(0)
    table = torch.randn(V, E, device=DEV, generator=g) * 0.02
    m, v = torch.zeros_like(table), torch.zeros_like(table)
    _, args = adam_args()
    own = ids_for(B, L, V, K, zipf=a.zipf)
    nown = own.shape[0]
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    base = {}
    pooled = torch.empty(nown, E, device=DEV)
    den = torch.empty(nown, device=DEV)
    base["gather_own_us"] = graph_us(lambda: call("tt_bag_mean_fwd", ptr(table), V, E, ptr(own), _lib.TT_IDS_I32, nown,
                                                  L, L, ptr(pooled), ptr(den), st()))
    d_pooled = torch.randn(nown, E, device=DEV, generator=g)
    p1 = ops.BagPlan(own, V, E, 0)
    p1.wait()
    base["update_own_us"] = graph_us(lambda: ops.bag_mean_backward_adamw_planned(d_pooled, None, p1, table, m, v, args))
    del p1
    for R in (a.ranks or (1, 2, 4, 8)):
        El = E // R
        ids = torch.cat([own] + [ids_for(B, L, V, K, seed=1000 * r, zipf=a.zipf) for r in range(1, R)]).contiguous()
        N = ids.shape[0]
        slab = table[:, :El].contiguous()
        ms, vs = torch.zeros_like(slab), torch.zeros_like(slab)
        part = torch.empty(N, El, device=DEV)
        den_all = torch.empty(N, device=DEV)
        res = {"config": shape, "ranks": R, "El": El, "tokens_per_rank": int((own > 0).sum())}
        res.update(base)
        res["col_gather_us"] = graph_us(lambda: call("tt_bag_mean_fwd_cols", ptr(slab), V, El, E, ptr(ids),
                                                     _lib.TT_IDS_I32, N, L, L, ptr(part), ptr(den_all), st()))
        res["col_gather_free_order_us"] = graph_us(lambda: call("tt_bag_mean_fwd", ptr(slab), V, El, ptr(ids),
                                                                _lib.TT_IDS_I32, N, L, L, ptr(part), ptr(den_all), st()))
        recv = torch.randn(N, El, device=DEV)
        out = torch.empty(nown, E, device=DEV)
        res["permute_pooled_us"] = graph_us(lambda: out.copy_(recv.view(R, nown, El).permute(1, 0, 2).reshape(nown, E)))
        gs = torch.randn(nown, E, device=DEV)
        send = torch.empty(N, El, device=DEV)
        res["permute_grad_us"] = graph_us(lambda: send.view(R, nown, El).copy_(gs.view(nown, R, El).permute(1, 0, 2)))
        segs, valss = [], []
        for r in range(R):
            pl = ops.BagPlan(ids[r * nown:(r + 1) * nown], V, El, 0)
            pl.wait()
            offs = (ctypes.c_int64 * 3)()
            call("tt_bag_plan_layout", pl.nseq, pl.L, V, El, offs)
            b0 = (-pl.buf.data_ptr()) % 256
            valss.append(pl.buf[b0 + offs[1]: b0 + offs[1] + 4 * nown * L].view(torch.int32).clone())
            segs.append(pl.buf[b0 + offs[2]: b0 + offs[2] + 4 * (V + 1)].view(torch.int32).clone())
            del pl
        seg_all, vals_all = torch.cat(segs), torch.cat(valss)
        gs_all = torch.randn(N, El, device=DEV, generator=g) * 1e-3
        nws = _lib.lib().tt_bag_col_reduce_ws_size(V, R, nown * L, El)
        cws = torch.empty(nws, dtype=torch.uint8, device=DEV)
        res["col_update_us"] = graph_us(lambda: call("tt_bag_col_reduce_ex", ptr(seg_all), ptr(vals_all), nown * L, R,
                                                     nown, ptr(gs_all), V, El, None, ptr(slab), ptr(ms), ptr(vs),
                                                     ptr(args), ptr(cws), nws, st()))
        # without the hot-row path (every row walked by one sub-wave: the round-5 kernel)
        if not a.no_serial:
            res["col_update_no_pieces_us"] = graph_us(lambda: call("tt_bag_col_reduce", ptr(seg_all), ptr(vals_all),
                                                                   nown * L, R, nown, ptr(gs_all), V, El, None,
                                                                   ptr(slab), ptr(ms), ptr(vs), ptr(args), st()))
        lens = torch.bincount(ids[ids > 0].long().flatten(), minlength=V)
        res["zipf"] = a.zipf
        res["hottest_row_tokens"] = int(lens.max())
        del cws
        res = {k: (round(x, 1) if isinstance(x, float) and k != "zipf" else x) for k, x in res.items()}
        res["link_MB_per_rank"] = {
            "ids_allgather": round((R - 1) * nown * L * 4 / 1e6, 1),
            "pooled_alltoall": round((R - 1) / R * nown * E * 4 / 1e6, 1),
            "grad_alltoall": round((R - 1) / R * nown * E * 4 / 1e6, 1),
            "plan_allgather_hidden": round((R - 1) * (nown * L + V + 1) * 4 / 1e6, 1)}
        print(json.dumps(res), flush=True)
        del ids, slab, ms, vs, part, recv, out, gs, send, seg_all, vals_all, gs_all, segs, valss
        torch.cuda.empty_cache()


def l2prep(a):
    """tt_inbatch_l2_prep alone (the head's normalise fused with the scorer's operand prep) at C3's
    rows (B = 8192 queries + 16384 candidates, H = 256, bf16), the B x B pairs form (8192 + 8192) and
    C2 (4096 + 8192, H = 128, fp32: the split engine's candidate planes), net of the copy that resets
    the rows: the pass's own cost without the concurrent sort plan of the step."""
    for B, M, H, name in ((8192, 16384, 256, "bf16"), (8192, 8192, 256, "bf16"), (4096, 8192, 128, "fp32")):
        dt = _lib.compute_dtype_code(name)
        y0 = torch.randn(B + M, H, device=DEV)
        y = y0.clone()
        norms = torch.empty(B + M, device=DEV)
        ws = torch.empty(_lib.lib().tt_inbatch_ws_size(B, M, H, dt), dtype=torch.uint8, device=DEV)

        def prep():  # the stream at call time: graph_us captures on a stream of its own
            y.copy_(y0)
            call("tt_inbatch_l2_prep", ptr(y), B, M, H, dt, ptr(norms), ptr(ws), ws.numel(),
                 torch.cuda.current_stream().cuda_stream)

        def copy_only():
            y.copy_(y0)

        t_prep, t_copy = graph_us(prep), graph_us(copy_only)
        out_b = 2 if name == "bf16" else 6  # the bf16 copy, or the fp32 scorer's three candidate planes
        print(json.dumps({"B": B, "M": M, "H": H, "dtype": name, "l2_prep_us": round(t_prep - t_copy, 1),
                          "copy_us": round(t_copy, 1), "bytes_MB": round((B + M) * H * (4 + 4 + out_b) / 1e6, 1)}),
              flush=True)


def scorer_once(a):
    B, M, H = int(a.shape), int(a.rest[0]), int(a.rest[1])
    dt = a.rest[2] if len(a.rest) > 2 else "bf16"
    g = torch.Generator(device=DEV).manual_seed(0)
    q = torch.nn.functional.normalize(torch.randn(B, H, device=DEV, generator=g), dim=-1).requires_grad_(True)
    d = torch.nn.functional.normalize(torch.randn(M, H, device=DEV, generator=g), dim=-1).requires_grad_(True)
    for _ in range(3):
        ops.in_batch_softmax_loss(q, d, 0.1, compute_dtype=dt).backward()
    torch.cuda.synchronize()


def next_rows(a):
    """each op's device time (graph replay), algorithmic bytes and the fraction of 8 TB/s,
    with the torch expression of the same result beside it."""
    out = {}
    peak = 8000.0

    def rec(name, us, nbytes, torch_us=None, **kw):
        e = {"us": round(us, 2), "algorithmic_MB": round(nbytes / 1e6, 2), "gbs": round(nbytes / us / 1e3, 1),
             "frac_of_8TBs": round(nbytes / us / 1e3 / peak, 3)}
        if torch_us is not None:
            e["torch_us"] = round(torch_us, 2)
        e.update(kw)
        out[name] = e
        print(name, json.dumps(e), flush=True)

    g = torch.Generator(device=DEV).manual_seed(0)
    # f1 device feeder: 500k resident int32 triplets of 64 tokens (384 MB), one C3 batch of 8192 by index
    N, L, B = 500_000, 64, 8192
    rows = torch.randint(1, 200_000, (3, N, L), device=DEV, dtype=torch.int32, generator=g)
    store = tt.data.DeviceTripletStore(rows)
    idx = torch.randperm(N, device=DEV, generator=g)[:B]
    buf = torch.empty(3 * B, L, dtype=torch.int32, device=DEV)
    rec("f1_feeder_gather", graph_us(lambda: store.gather(idx, out=buf), 20), 2 * 3 * B * L * 4 + B * 8,
        graph_us(lambda: rows.index_select(1, idx), 20), shape=f"(3, {N}, {L}) int32 store, batch {B}")
    del rows, store
    # f2 forward-only encode (C3 tower, no grad): bag gather + head + F.normalize over 8192 documents
    V, E = 200_000, 256
    emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
    model = tt.build_two_tower("mean", emb, hidden_dim=E, tied_weights=True).to(DEV).eval()
    ids = tt.data.synthetic_triplets(B, L, V, seed=3, device=DEV)[1]
    nnz = int((ids > 0).sum())
    with torch.no_grad():
        us = graph_us(lambda: model.encode_document(ids), 10)
    rec("f2_encode_documents", us, ids.numel() * ids.element_size() + nnz * E * 4 + B * E * 4 * 3,
        docs_per_s=round(B / us * 1e6), note="bytes: ids + gathered rows + pooled, h, y rows (head MFMA-bound)")
    # f2 cosine scores over a 1M x 256 index, top-k of each query's row
    ND = 1_000_000
    docs = torch.nn.functional.normalize(torch.randn(ND, E, device=DEV, generator=g), dim=-1)
    for nq in (1, 8, 16, 32, 64):
        q = torch.randn(nq, E, device=DEV, generator=g)
        dn = docs.norm(dim=1)
        t_us = graph_us(lambda: (q @ docs.t()) / (q.norm(dim=1, keepdim=True) * dn).clamp_min(1e-8), 10)
        rec(f"f2_cosine_scores_nq{nq}", graph_us(lambda: ops.cosine_scores(q, docs), 10),
            ND * E * 4 + nq * ND * 4 + nq * E * 4, t_us, note="torch: mm / norms (not the ATen eps form)")
        sc = ops.cosine_scores(q, docs)
        for k in (10, 100):
            rec(f"f2_topk_nq{nq}_k{k}", graph_us(lambda: ops.topk_rows(sc, k), 10), nq * ND * 4 + nq * k * 12,
                graph_us(lambda: torch.topk(sc, k, dim=1), 10))
    del docs
    # f4 AveragePoolingTower head at C3 rows (3 x 8192): projection 256 -> 128, LayerNorm + L2, fwd + bwd
    R, H = 3 * B, 128
    x = torch.randn(R, E, device=DEV, generator=g)
    W = torch.randn(H, E, device=DEV, generator=g) / 16
    b, gam, bet = (torch.randn(H, device=DEV, generator=g) for _ in range(3))
    hproj = ops.linear(x, W, b)
    dy = torch.randn(R, H, device=DEV, generator=g)
    rec("f4_linear_fwd", graph_us(lambda: ops.linear(x, W, b), 20), R * E * 4 + R * H * 4,
        graph_us(lambda: torch.addmm(b, x, W.t()), 20), note="split-bf16 MFMA, fp32 accuracy; torch: hipBLASLt fp32")
    rec("f4_ln_l2_fwd", graph_us(lambda: ops.layernorm_l2_normalize(hproj, gam, bet, 1e-5), 20),
        R * H * 4 * 2 + R * 12, graph_us(lambda: torch.nn.functional.normalize(
            torch.nn.functional.layer_norm(hproj, (H,), gam, bet, 1e-5), dim=-1), 20))
    # backward launches called directly (autograd's own host time left out; graph replay)
    stats = torch.empty(R, 3, device=DEV)
    yv = torch.empty_like(hproj)
    call("tt_ln_l2_fwd", ptr(hproj), R, H, ptr(gam), ptr(bet), 1e-5, ptr(yv), ptr(stats),
         torch.cuda.current_stream().cuda_stream)
    dxl, gx, gb = (torch.empty_like(hproj) for _ in range(3))

    def ln_bwd_unfolded():
        call("tt_ln_l2_bwd", ptr(dy), ptr(hproj), R, H, ptr(gam), ptr(bet), ptr(stats), ptr(dxl), ptr(gx), ptr(gb),
             torch.cuda.current_stream().cuda_stream)
        return ops.colsum(gx), ops.colsum(gb)

    dg, dbt = torch.empty(H, device=DEV), torch.empty(H, device=DEV)
    wsl = torch.empty(_lib.lib().tt_ln_l2_bwd_ws_size(R, H), dtype=torch.uint8, device=DEV)

    def ln_bwd():
        call("tt_ln_l2_bwd_ex", ptr(dy), ptr(hproj), R, H, ptr(gam), ptr(bet), ptr(stats), ptr(dxl), ptr(dg),
             ptr(dbt), ptr(wsl), wsl.numel(), torch.cuda.current_stream().cuda_stream)

    rec("f4_ln_l2_bwd", graph_us(ln_bwd, 20), R * H * 4 * 3 + R * 12 + 2 * H * 4,
        graph_us(ln_bwd_unfolded, 20), note="dx + dgamma, dbeta folded per workgroup, then column-summed (tt_ln_l2_bwd_ex); "
        "torch_us column: the per-row terms written out + two tt_colsum launches (round 4 form)")
    PWt = ops._planes(W, True)

    def lin_bwd():
        dx = ops._head_gemm(dy, PWt, 3, N=E)
        return dx, ops.head_wgrad(dy, x)

    rec("f4_linear_bwd", graph_us(lin_bwd, 20), R * H * 4 * 2 + R * E * 4 * 2 + H * E * 4,
        note="dx (tt_head_gemm epi 3) + dW, db (tt_head_wgrad_ex)")
    # a6 triplet loss (losses.py:9-44) at C3 rows: forward + backward kernels against the reference's
    # torch expression (F.cosine_similarity, relu, mean) forward + backward
    Bt, Ht = 8192, 256
    qt_, pt_, nt_ = (torch.randn(Bt, Ht, device=DEV, generator=g) for _ in range(3))
    dq_, dp_, dn_ = (torch.empty(Bt, Ht, device=DEV) for _ in range(3))
    gl = torch.ones(1, device=DEV)

    def trip():
        ops._triplet_fwd(qt_, pt_, nt_, 0.2)
        ops._triplet_bwd(qt_, pt_, nt_, 0.2, gl, dq_, dp_, dn_)

    qr, pr, nr = (t.clone().requires_grad_(True) for t in (qt_, pt_, nt_))

    def trip_torch():
        F = torch.nn.functional
        loss = F.relu(0.2 - F.cosine_similarity(qr, pr, dim=1) + F.cosine_similarity(qr, nr, dim=1)).mean()
        return torch.autograd.grad(loss, (qr, pr, nr))

    rec("a6_triplet_fwd_bwd", graph_us(trip, 20), Bt * Ht * 4 * 6, event_us(trip_torch, 20),
        note="reads q, p, n twice (fwd, bwd), writes dq, dp, dn; torch_us: eager autograd of the reference expression")
    path = a.shape
    if path:
        with open(path, "w") as f:
            json.dump(out, f, indent=1)


def search_once(a):
    """Cosine scores of 1 and of 64 queries over a 1M x 256 index and the top 10 of each row, five
    times each, nothing else (counter passes: tools/profile_mb.sh)."""
    g = torch.Generator(device=DEV).manual_seed(0)
    docs = torch.randn(1_000_000, 256, device=DEV, generator=g)
    for nq in (1, 64):
        q = torch.randn(nq, 256, device=DEV, generator=g)
        for _ in range(5):
            ops.topk_rows(ops.cosine_scores(q, docs), 10)
    torch.cuda.synchronize()


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("what", choices=["bag_bwd", "plan", "head", "scorer", "scorer_dp", "split_fwd", "table_sync",
                                     "column_sync", "l2prep", "scorer_once", "next_rows",
                                     "search_once"])
    ap.add_argument("shape", nargs="?", default=None)
    ap.add_argument("rest", nargs="*")
    ap.add_argument("--zipf", type=float, default=None)
    ap.add_argument("--ranks", type=int, nargs="*", default=None, help="column_sync: only these rank counts")
    ap.add_argument("--no-serial", action="store_true", help="column_sync: skip the round-5 serial-row timing")
    a = ap.parse_args()
    if a.what == "scorer_once" and len(a.rest) > 3:  # a variant library (tools/build_variants.sh)
        _lib.LIB_PATH = os.path.abspath(a.rest[3])
    if a.what == "scorer" and a.shape is not None:
        a.rest = [a.shape] + a.rest
    globals()[a.what](a)


if __name__ == "__main__":
    main()
