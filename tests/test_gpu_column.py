"""Column-sharded table kernels (table_sync "column", distributed.ColumnTable), simulated on one GPU:
W "ranks" each sort their own sequences (tt_bag_plan), the plans are concatenated as the all-gather
would deliver them, and tt_bag_col_reduce forms the gradient of each rank's column slab from every
rank's tokens.  Checked against the float64 oracle's dense table gradient of the global batch
(oracle.reference_math.bag_mean_bwd: embeddings.py:30 via train.py:138) at 1e-5, and bit for bit
against the single-plan reduce of the concatenated batch at the same columns (tt_bag_mean_bwd_planned:
the merged per-source order and interleaved partial sums are the same, and with the hot-row path,
tt_bag_col_reduce_ex, so are the pieces of rows up to 32,768 merged tokens), and the fused AdamW form
against tt_bag_mean_bwd_adamw_planned likewise."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import reference_math as O
from twotower_amd import _lib, ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _plan_arrays(ids: torch.Tensor, V: int, El: int):
    """(seg (V + 1,), vals (nseq * L,)) int32 views of a local BagPlan, as ColumnPlan.exchange sends them."""
    plan = ops.BagPlan(ids, V, El, 0)
    plan.wait()
    offs = (ctypes.c_int64 * 3)()
    ops.call("tt_bag_plan_layout", plan.nseq, plan.L, plan.V, plan.E, offs)
    base = (-plan.buf.data_ptr()) % 256
    n = plan.nseq * plan.L
    vals = plan.buf[base + offs[1]: base + offs[1] + 4 * n].view(torch.int32)
    seg = plan.buf[base + offs[2]: base + offs[2] + 4 * (V + 1)].view(torch.int32)
    return seg.clone(), vals.clone()


def _ids(rng, kind, V, n, L):
    """uniform ids; Zipf(1.05) ids (the hottest rows hold a few % of all tokens);
    "char": a 34-row character vocabulary (tokenisers.py:50,59: every row is a hot row); "hot": 60 %
    of the tokens on one row (a row past kPieceT * kMaxPieces merged tokens: the group level)."""
    if kind == "zipf":
        return np.minimum(rng.zipf(1.05, size=(n, L)), V - 1)
    if kind == "hot":
        ids = rng.integers(1, V, size=(n, L))
        ids[rng.random((n, L)) < 0.6] = 5
        return ids
    return rng.integers(0, V, size=(n, L))


def _setup(W, E, V, nseq, L, seed, kind="uniform"):
    rng = np.random.default_rng(seed)
    ids = _ids(rng, kind, V, W * nseq, L)
    ids[np.arange(L)[None, :] >= rng.integers(0, L + 1, size=W * nseq)[:, None]] = 0  # ragged
    ids[0, :] = 0                      # an all-padding sequence
    ids[1, :] = V - 1                  # the last row, repeated
    ids_t = torch.as_tensor(ids, dtype=torch.int32, device=DEV)
    gs = torch.as_tensor(rng.standard_normal((W * nseq, E)).astype(np.float32), device=DEV)
    El = E // W
    segs, valss = zip(*(_plan_arrays(ids_t[s * nseq:(s + 1) * nseq], V, El) for s in range(W)))
    return ids, ids_t, gs, torch.cat(segs), torch.cat(valss)


@pytest.mark.parametrize("W,E", [(1, 256), (2, 256), (4, 256), (8, 256), (2, 64), (4, 128), (8, 512)])
def test_column_reduce_equals_single_plan_and_oracle(W, E):
    V, nseq, L = 3001, 96, 40
    if E // W not in (32, 64, 128, 256):
        pytest.skip("slab width outside the column kernels")
    El = E // W
    ids, ids_t, gs, seg_all, vals_all = _setup(W, E, V, nseq, L, seed=W * 1000 + E)
    # single plan over the concatenated batch, full width (denom None: gs already scaled)
    whole = ops.bag_mean_backward_planned(gs, None, ops.BagPlan(ids_t, V, E, 0))
    oracle = O.bag_mean_bwd(gs.double().cpu().numpy(), np.ones(W * nseq), ids, V, 0)
    for c in range(W):
        gs_all = gs[:, c * El:(c + 1) * El].contiguous()
        grad = torch.empty(V, El, device=DEV)
        ops.call("tt_bag_col_reduce", seg_all.data_ptr(), vals_all.data_ptr(), nseq * L, W, nseq, gs_all.data_ptr(), V,
                 El, grad.data_ptr(), None, None, None, None, _lib.stream_of(grad))
        want = whole[:, c * El:(c + 1) * El]
        assert torch.equal(grad, want), (c, float((grad - want).abs().max()))
        o = oracle[:, c * El:(c + 1) * El]
        assert np.abs(grad.double().cpu().numpy() - o).max() / np.abs(o).max() < 1e-5


def _col_reduce_ex(seg_all, vals_all, nL, W, nseq, gs_all, V, El, grad=None, slab=None, m=None, v=None, args=None):
    n = _lib.lib().tt_bag_col_reduce_ws_size(V, W, nL, El)
    ws = torch.empty(n, dtype=torch.uint8, device=DEV)
    p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    ops.call("tt_bag_col_reduce_ex", seg_all.data_ptr(), vals_all.data_ptr(), nL, W, nseq, gs_all.data_ptr(), V, El,
             p(grad), p(slab), p(m), p(v), p(args), ws.data_ptr(), n, _lib.stream_of(gs_all))


@pytest.mark.parametrize("kind,V", [("zipf", 3001), ("char", 34), ("uniform", 3001)])
@pytest.mark.parametrize("W", [2, 4, 8])
def test_column_reduce_hot_rows(kind, V, W):
    """The hot-row path (tt_bag_col_reduce_ex: rows of more than 128 merged tokens summed in pieces,
    one sub-wave each, then folded) under Zipf(1.05) ids and C1's 34-row character vocabulary, at
    W = 2 / 4 / 8 (El 128 / 64 / 32): every row is at most 32,768 merged tokens here, where the piece
    partition is the single plan's, so the gradient equals the single-plan reduce of the concatenated
    batch bit for bit, and the float64 oracle's dense table gradient at 1e-5; the fused AdamW form
    equals tt_bag_mean_bwd_adamw_planned bit for bit."""
    E, nseq, L = 256, 192, 40
    El = E // W
    ids, ids_t, gs, seg_all, vals_all = _setup(W, E, V, nseq, L, seed=31 * W + V, kind=kind)
    lens = np.bincount(ids[ids > 0].ravel(), minlength=V)
    if kind != "uniform":
        assert lens.max() > 128  # the piece path runs
    assert lens.max() <= 128 * 256
    whole = ops.bag_mean_backward_planned(gs, None, ops.BagPlan(ids_t, V, E, 0))
    oracle = O.bag_mean_bwd(gs.double().cpu().numpy(), np.ones(W * nseq), ids, V, 0)
    rng = np.random.default_rng(3)
    tbl = torch.as_tensor(rng.standard_normal((V, E)).astype(np.float32), device=DEV)
    m = torch.as_tensor(rng.standard_normal((V, E)).astype(np.float32) * 0.01, device=DEV)
    v = torch.as_tensor(np.abs(rng.standard_normal((V, E))).astype(np.float32) * 1e-4, device=DEV)
    step = torch.tensor(3.0, device=DEV)
    args = torch.zeros(8, device=DEV)
    ops.adam_prepare([(step, args)], lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01)
    t1, m1, v1 = tbl.clone(), m.clone(), v.clone()
    ops.bag_mean_backward_adamw_planned(gs, None, ops.BagPlan(ids_t, V, E, 0), t1, m1, v1, args)
    for c in range(W):
        sl = slice(c * El, (c + 1) * El)
        gs_all = gs[:, sl].contiguous()
        grad = torch.empty(V, El, device=DEV)
        _col_reduce_ex(seg_all, vals_all, nseq * L, W, nseq, gs_all, V, El, grad=grad)
        torch.cuda.synchronize()
        assert torch.equal(grad, whole[:, sl]), (c, float((grad - whole[:, sl]).abs().max()))
        o = oracle[:, sl]
        assert np.abs(grad.double().cpu().numpy() - o).max() / np.abs(o).max() < 1e-5
        ts, ms, vs = tbl[:, sl].contiguous(), m[:, sl].contiguous(), v[:, sl].contiguous()
        _col_reduce_ex(seg_all, vals_all, nseq * L, W, nseq, gs_all, V, El, slab=ts, m=ms, v=vs, args=args)
        torch.cuda.synchronize()
        assert torch.equal(ts, t1[:, sl]) and torch.equal(ms, m1[:, sl]) and torch.equal(vs, v1[:, sl]), c


@pytest.mark.parametrize("W", [2, 8])
def test_column_reduce_row_past_single_plan_pieces(W):
    """A row of more than 128 x 256 merged tokens (60 % of a global batch on one row): up to 4,096
    pieces and the group level (groups of 256 piece partials), against the float64 oracle at 1e-5
    (the single plan cuts such a row into 256 longer pieces, so the sums associate differently)."""
    E, V, nseq, L = 256, 3001, 4096 // W, 64
    El = E // W
    ids, ids_t, gs, seg_all, vals_all = _setup(W, E, V, nseq, L, seed=77 + W, kind="hot")
    lens = np.bincount(ids[ids > 0].ravel(), minlength=V)
    assert lens.max() > 128 * 256
    oracle = O.bag_mean_bwd(gs.double().cpu().numpy(), np.ones(W * nseq), ids, V, 0)
    for c in (0, W - 1):
        sl = slice(c * El, (c + 1) * El)
        gs_all = gs[:, sl].contiguous()
        grad = torch.empty(V, El, device=DEV)
        _col_reduce_ex(seg_all, vals_all, nseq * L, W, nseq, gs_all, V, El, grad=grad)
        torch.cuda.synchronize()
        o = oracle[:, sl]
        err = np.abs(grad.double().cpu().numpy() - o).max() / np.abs(o).max()
        assert err < 1e-5, (c, float(err))
        # and the row-without-pieces path is unchanged: the old entry walks the hot row serially
        g0 = torch.empty(V, El, device=DEV)
        ops.call("tt_bag_col_reduce", seg_all.data_ptr(), vals_all.data_ptr(), nseq * L, W, nseq, gs_all.data_ptr(), V,
                 El, g0.data_ptr(), None, None, None, None, _lib.stream_of(g0))
        torch.cuda.synchronize()
        cold = lens <= 128
        assert torch.equal(grad[torch.as_tensor(cold, device=DEV)], g0[torch.as_tensor(cold, device=DEV)])


@pytest.mark.parametrize("W,E", [(2, 256), (8, 256), (2, 128)])
def test_column_adamw_equals_fused_planned(W, E):
    V, nseq, L = 3001, 96, 40
    El = E // W
    ids, ids_t, gs, seg_all, vals_all = _setup(W, E, V, nseq, L, seed=7 + W)
    rng = np.random.default_rng(5)
    tbl = torch.as_tensor(rng.standard_normal((V, E)).astype(np.float32), device=DEV)
    m = torch.as_tensor(rng.standard_normal((V, E)).astype(np.float32) * 0.01, device=DEV)
    v = torch.as_tensor(np.abs(rng.standard_normal((V, E))).astype(np.float32) * 1e-4, device=DEV)
    step = torch.tensor(2.0, device=DEV)
    args = torch.zeros(8, device=DEV)
    ops.adam_prepare([(step, args)], lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01)
    t1, m1, v1 = tbl.clone(), m.clone(), v.clone()
    ops.bag_mean_backward_adamw_planned(gs, None, ops.BagPlan(ids_t, V, E, 0), t1, m1, v1, args)
    for c in range(W):
        sl = slice(c * El, (c + 1) * El)
        ts, ms, vs = tbl[:, sl].contiguous(), m[:, sl].contiguous(), v[:, sl].contiguous()
        gs_all = gs[:, sl].contiguous()
        ops.call("tt_bag_col_reduce", seg_all.data_ptr(), vals_all.data_ptr(), nseq * L, W, nseq, gs_all.data_ptr(), V,
                 El, None, ts.data_ptr(), ms.data_ptr(), vs.data_ptr(), args.data_ptr(), _lib.stream_of(ts))
        assert torch.equal(ts, t1[:, sl]) and torch.equal(ms, m1[:, sl]) and torch.equal(vs, v1[:, sl]), c


def test_bag_forward_slab_32_columns():
    """tt_bag_mean_fwd at E = 32 (a 256-wide table's column slab over 8 ranks) against the oracle."""
    rng = np.random.default_rng(9)
    V, N, L = 5000, 300, 64
    ids = rng.integers(0, V, size=(N, L))
    ids[np.arange(L)[None, :] >= rng.integers(0, L + 1, size=N)[:, None]] = 0
    ids[0, :] = 0
    tbl = rng.standard_normal((V, 32)).astype(np.float32)
    pooled, denom = ops.bag_mean_forward(torch.as_tensor(tbl, device=DEV), torch.as_tensor(ids, device=DEV))
    want, wden = O.bag_mean_fwd(tbl, ids)
    assert np.abs(pooled.double().cpu().numpy() - want).max() / np.abs(want).max() < 1e-6
    assert np.array_equal(denom.cpu().numpy(), wden.astype(np.float32))
    # single-token bags reproduce table rows exactly (the gather is bit-exact)
    one = np.zeros((64, L), dtype=np.int64)
    one[:, 0] = rng.integers(1, V, size=64)
    p1, _ = ops.bag_mean_forward(torch.as_tensor(tbl, device=DEV), torch.as_tensor(one, device=DEV))
    assert np.array_equal(p1.cpu().numpy(), (tbl[one[:, 0]] / np.float32(1.0 + 1e-9)).astype(np.float32))


@pytest.mark.parametrize("E,El", [(256, 32), (256, 64), (256, 128), (256, 256), (128, 32), (128, 64), (64, 32),
                                  (512, 64)])
@pytest.mark.parametrize("L", [64, 100, 7])
def test_column_slab_forward_equals_full_width_bits(E, El, L):
    """tt_bag_mean_fwd_cols over each column slab of a table equals tt_bag_mean_fwd at the full width
    on those columns bit for bit (the pooled rows a column-sharded step assembles are the one-GPU
    forward's), with ragged / padded / out-of-range ids and L past one 64-token chunk; int32 and
    int64 ids."""
    rng = np.random.default_rng(E + El + L)
    V, N = 3000, 777
    ids = rng.integers(0, V + 3, size=(N, L))  # a few ids >= V: masked, as the full-width gather does
    ids[np.arange(L)[None, :] >= rng.integers(0, L + 1, size=N)[:, None]] = 0
    ids[0, :] = 0
    ids[1, :] = V - 1
    tbl = torch.as_tensor(rng.standard_normal((V, E)).astype(np.float32), device=DEV)
    for dt in (torch.int64, torch.int32):
        idt = torch.as_tensor(ids, device=DEV).to(dt)
        full, fden = ops.bag_mean_forward(tbl, idt)
        for c0 in range(0, E, El):
            slab = tbl[:, c0:c0 + El].contiguous()
            part = torch.empty(N, El, device=DEV)
            den = torch.empty(N, device=DEV)
            ops.call("tt_bag_mean_fwd_cols", slab.data_ptr(), V, El, E, idt.data_ptr(), _lib.ids_dtype_code(idt), N, L,
                     L, part.data_ptr(), den.data_ptr(), _lib.stream_of(slab))
            torch.cuda.synchronize()
            assert torch.equal(part, full[:, c0:c0 + El]), (dt, c0)
            assert torch.equal(den, fden)
