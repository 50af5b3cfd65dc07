"""Autograd wrappers over the C ABI.  Every forward/backward here launches HIP kernels from
libtwotower_amd.so on the tensor's current stream; nothing falls back to ATen compute.

Reference call sites each op replaces are cited per function (paths inside k0r1g/two-towers).
"""
from __future__ import annotations

import contextlib
import ctypes
import functools
import os

import torch

from . import _lib
from ._lib import call, ptr, require_gpu, stream_of

_FLOAT = torch.float32


def _contig_f32(t: torch.Tensor, name: str) -> torch.Tensor:
    if t.dtype != _FLOAT:
        raise TypeError(f"{name} must be float32, got {t.dtype}")
    return t.contiguous()


# --------------------------------------------------------------------------------------------
# Embedding bag: gather + masked mean-pool   (twotower/embeddings.py:30,40; encoders.py:62-72)
class _Workspace:
    """Per-device scratch buffers grown on demand (the C side never allocates)."""

    def __init__(self):
        self._bufs: dict[tuple, torch.Tensor] = {}

    def get(self, key: str, nbytes: int, device: torch.device) -> torch.Tensor:
        k = (key, device)
        buf = self._bufs.get(k)
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=device)
            self._bufs[k] = buf
        return buf


WORKSPACE = _Workspace()


def bag_mean_forward(weight: torch.Tensor, ids: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """pooled (N, E) and denom (N,) = count of ids > 0 plus 1e-9 (encoders.py:62-72)."""
    require_gpu(weight, ids)
    if ids.dim() != 2:
        raise ValueError(f"ids must be (batch, seq_len), got shape {tuple(ids.shape)}")
    ids = ids.contiguous()
    V, E = weight.shape
    N, L = ids.shape
    pooled = torch.empty(N, E, dtype=_FLOAT, device=weight.device)
    denom = torch.empty(N, dtype=_FLOAT, device=weight.device)
    req = _PLANES_REQ[-1] if _PLANES_REQ else None
    if req is not None and req[0].shape[1] == E and req[0].device == weight.device:
        # the consuming head's weight planes, formed by extra workgroups of this launch
        W1, W2 = req
        H = W1.shape[0]
        n1, n2 = _head_planes_bytes(E, H)
        planes = torch.empty(2 * (n1 + n2), dtype=torch.uint8, device=weight.device)  # W1, W2, W1^T, W2^T
        call("tt_bag_mean_fwd_split", ptr(weight), V, E, ptr(ids), _lib.ids_dtype_code(ids), N, L, L, ptr(pooled),
             ptr(denom), ptr(W1), ptr(W2), H, ptr(planes), stream_of(weight))
        _PLANES_REQ[-1] = None  # one gather per request
        _PLANES_DONE[(W1.data_ptr(), W2.data_ptr())] = planes
        return pooled, denom
    call("tt_bag_mean_fwd", ptr(weight), V, E, ptr(ids), _lib.ids_dtype_code(ids), N, L, L, ptr(pooled), ptr(denom),
         stream_of(weight))
    return pooled, denom


_PLANES_REQ: list = []  # (W1, W2) whose planes the next bag gather forms (open head_planes_in_gather), or None
_PLANES_DONE: dict = {}  # (W1, W2 data_ptr) -> planes that gather formed, taken by that head's TowerHead


@functools.lru_cache(maxsize=None)
def _head_planes_bytes(E: int, H: int) -> tuple[int, int]:
    return _lib.lib().tt_head_planes_bytes(H, E), _lib.lib().tt_head_planes_bytes(H, H)


@contextlib.contextmanager
def head_planes_in_gather(W1: torch.Tensor, W2: torch.Tensor):
    """While open, the next bag gather whose rows feed the tower head (W1, W2) also forms that
    head's weight planes in its own launch (tt_bag_mean_fwd_split), and the head takes them
    instead of launching tt_head_split_ff2 between the gather and its first GEMM (C3: that
    launch sat on the step's critical path for 9-15 us).  The encoders open it around a
    MeanPoolingTower's gather and head.  TT_PLANES_IN_GATHER=0 turns it off.  (Splitting on a
    side stream before the gather instead was measured slower: +6 us on the plan's stream, +27 us
    on a stream of its own -- the cross-queue wait in the replayed graph costs more than the
    split; profiles/r03zf_planes_ab.txt.)"""
    on = (os.environ.get("TT_PLANES_IN_GATHER", "1") != "0" and W1.is_cuda and W1.dtype == _FLOAT
          and W2.dtype == _FLOAT and W1.is_contiguous() and W2.is_contiguous() and W1.shape[1] in EMB_WIDTHS
          and W1.shape[0] in HEAD_WIDTHS and tuple(W2.shape) == (W1.shape[0], W1.shape[0]))
    _PLANES_REQ.append((W1, W2) if on else None)
    key = (W1.data_ptr(), W2.data_ptr())
    try:
        yield
    finally:
        _PLANES_REQ.pop()
        _PLANES_DONE.pop(key, None)


def bag_mean_backward(d_pooled: torch.Tensor, denom: torch.Tensor, ids: torch.Tensor, V: int,
                      padding_idx: int | None, mode: int = _lib.TT_SCATTER_SORTED) -> torch.Tensor:
    """Dense (V, E) table gradient (embedding_dense_backward of the pooled lookup)."""
    d_pooled = _contig_f32(d_pooled, "d_pooled")
    N, E = d_pooled.shape
    L = ids.shape[1]
    dev = d_pooled.device
    pad = -1 if padding_idx is None else int(padding_idx)
    if mode == _lib.TT_SCATTER_ATOMIC:
        grad = torch.zeros(V, E, dtype=_FLOAT, device=dev)
        call("tt_bag_mean_bwd", ptr(d_pooled), ptr(denom), ptr(ids), _lib.ids_dtype_code(ids), N, L, L, V, E, pad,
             ptr(grad), mode, None, 0, stream_of(d_pooled))
        return grad
    grad = torch.empty(V, E, dtype=_FLOAT, device=dev)
    nbytes = _lib.lib().tt_bag_mean_bwd_ws_size(N, L, V, E)
    ws = WORKSPACE.get("bag_bwd", nbytes, dev)
    call("tt_bag_mean_bwd", ptr(d_pooled), ptr(denom), ptr(ids), _lib.ids_dtype_code(ids), N, L, L, V, E, pad,
         ptr(grad), mode, ptr(ws), ws.numel(), stream_of(d_pooled))
    return grad


class BagPlan:
    """The id-only half of the sorted backward (tt_bag_plan), launched on the side stream as soon
    as the forward has its ids, so its radix sort runs beside the towers and the scorer.  The
    backward (or the fused optimizer) waits on ``ready`` before using it."""

    __slots__ = ("ids", "buf", "ready", "nseq", "L", "V", "E", "pad")

    def __init__(self, ids: torch.Tensor, V: int, E: int, padding_idx: int | None, gather_group=None):
        """gather_group: data parallel with a replicated table update -- the plan covers the ids
        of every rank (all-gathered here, on the side stream, rank-major)."""
        dev = ids.device
        self.V, self.E = V, E
        main = torch.cuda.current_stream(dev)
        side = _lib.side_stream(dev)
        side.wait_stream(main)
        ids.record_stream(side)  # allocated on the current stream, read on the side stream
        self.pad = -1 if padding_idx is None else int(padding_idx)
        with torch.cuda.stream(side):
            if gather_group is not None:
                from .distributed import all_gather_rows

                world = torch.distributed.get_world_size(gather_group)
                ids_all = ids.new_empty((world * ids.shape[0],) + tuple(ids.shape[1:]))
                all_gather_rows(ids_all, ids, gather_group)
                ids = ids_all
            self.ids = ids
            self.nseq, self.L = ids.shape
            nbytes = _lib.lib().tt_bag_plan_ws_size(self.nseq, self.L, V, E)
            self.buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            call("tt_bag_plan", ptr(ids), _lib.ids_dtype_code(ids), self.nseq, self.L, self.L, V, E, self.pad,
                 ptr(self.buf), self.buf.numel(), side.cuda_stream)
        self.ready = torch.cuda.Event()
        self.ready.record(side)

    def wait(self) -> None:
        cur = torch.cuda.current_stream(self.buf.device)
        cur.wait_event(self.ready)
        self.buf.record_stream(cur)  # allocated on the side stream, read here


def plan_fork_early(table_bytes: int) -> bool:
    """Whether the tower bag's sort forks before its gather (see BagMeanPool.forward).
    TT_PLAN_FORK: "auto" (default) forks before the gather inside a graph capture when the table
    fits the 256 MiB Infinity Cache, and after it otherwise and in every eager step: an eager step
    that starts on an idle GPU (the reference loop's .item() syncs) then does not queue its gather
    behind the sort's host launches (C3 reference loop with both opt-ins, same box, 5 runs each:
    1.107-1.149 against 1.136-1.204 ms/step, profiles/r05zl_plain_fork_ab.txt).  "size" applies the
    table-size rule in eager steps too; "early" and "late" force one side."""
    mode = os.environ.get("TT_PLAN_FORK", "auto")
    if mode in ("early", "late"):
        return mode == "early"
    if mode == "auto" and not torch.cuda.is_current_stream_capturing():
        return False
    return table_bytes <= 256 * 2 ** 20


class _BagGradToken:
    """Shared by a BagMeanPool node and the TowerHead that is the sole consumer of its output:
    the head's dx GEMM divides each row by its bag denominator in its epilogue (tt_head_gemm epi
    5) and leaves the result here, so the bag backward skips its scaling pass."""

    __slots__ = ("denom", "grad")

    def __init__(self, denom: torch.Tensor):
        self.denom, self.grad = denom, None


_SOLE_HEAD: list = []  # pooled tensors whose only consumer is the TowerHead about to run


@contextlib.contextmanager
def bag_head_prescale(pooled: torch.Tensor):
    """While open, a TowerHead applied to ``pooled`` (the output of bag_mean_pool, consumed by
    nothing else: the encoders' own forward paths open it) forms the bag backward's
    d_pooled / denom in its dx epilogue.  TT_BAG_PRESCALE=0 turns it off."""
    tok = getattr(pooled, "_tt_bag_token", None)
    on = tok is not None and os.environ.get("TT_BAG_PRESCALE", "1") != "0"
    _SOLE_HEAD.append(pooled if on else None)
    try:
        yield
    finally:
        _SOLE_HEAD.pop()


def bag_mean_backward_planned(d_pooled: torch.Tensor, denom: torch.Tensor, plan: BagPlan,
                              out: torch.Tensor | None = None) -> torch.Tensor:
    """Dense (V, E) table gradient from a BagPlan (every row written), into `out` if given."""
    d_pooled = _contig_f32(d_pooled, "d_pooled")
    plan.wait()
    grad = torch.empty(plan.V, plan.E, dtype=_FLOAT, device=d_pooled.device) if out is None else out
    if tuple(grad.shape) != (plan.V, plan.E) or not grad.is_contiguous() or grad.dtype != _FLOAT:
        raise ValueError("out must be a contiguous float32 (V, E) tensor")
    call("tt_bag_mean_bwd_planned", ptr(d_pooled), ptr(denom), plan.nseq, plan.L, plan.V, plan.E, ptr(plan.buf),
         plan.buf.numel(), ptr(grad), stream_of(d_pooled))
    return grad


def bag_mean_backward_planned_prepare(d_pooled: torch.Tensor, denom: torch.Tensor | None, plan: BagPlan) -> None:
    """First half of a row-range table gradient (tt_bag_mean_bwd_planned_prepare): the scaled rows
    and the long rows' piece sums, into the plan workspace; then bag_mean_backward_planned_rows."""
    d_pooled = _contig_f32(d_pooled, "d_pooled")
    plan.wait()
    call("tt_bag_mean_bwd_planned_prepare", ptr(d_pooled), ptr(denom), plan.nseq, plan.L, plan.V, plan.E,
         ptr(plan.buf), plan.buf.numel(), stream_of(d_pooled))


def bag_mean_backward_planned_rows(d_pooled: torch.Tensor, denom: torch.Tensor | None, plan: BagPlan, row_begin: int,
                                   row_end: int, out: torch.Tensor) -> torch.Tensor:
    """Rows [row_begin, row_end) of the dense table gradient into `out` ((row_end - row_begin, E)
    contiguous float32), after bag_mean_backward_planned_prepare on the same stream."""
    d_pooled = _contig_f32(d_pooled, "d_pooled")
    if tuple(out.shape) != (row_end - row_begin, plan.E) or not out.is_contiguous() or out.dtype != _FLOAT:
        raise ValueError("out must be a contiguous float32 (row_end - row_begin, E) tensor")
    call("tt_bag_mean_bwd_planned_rows", ptr(d_pooled), ptr(denom), plan.nseq, plan.L, plan.V, plan.E, ptr(plan.buf),
         plan.buf.numel(), int(row_begin), int(row_end), ptr(out), stream_of(d_pooled))
    return out


class DeferredTableGrad:
    """Table gradient kept in its factored form (ids, d_pooled, denom, plan) so a fused optimizer
    can apply scatter + AdamW in one pass (tt_bag_mean_bwd_adamw) without the dense V x E buffer.
    gather_group: data parallel, replicated table update (the plan covers every rank's ids).
    on_backward: a callable queued to run once at the end of each backward pass that produced
    parts (optim.BackwardTableUpdate: the fused update inside loss.backward(), for a loop that
    keeps torch.optim.AdamW)."""

    __slots__ = ("parts", "padding_idx", "gather_group", "on_backward", "queued")

    def __init__(self, padding_idx: int | None = 0, gather_group=None, on_backward=None):
        self.parts: list[tuple] = []
        self.padding_idx = padding_idx
        self.gather_group = gather_group
        self.on_backward = on_backward
        self.queued = False

    def added(self) -> None:
        """A backward node appended its part: queue on_backward for the end of this backward pass
        (once, however many bag calls on the table the pass differentiates)."""
        if self.on_backward is not None and not self.queued:
            self.queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._fire)

    def _fire(self) -> None:
        self.queued = False
        self.on_backward()


class BagMeanPool(torch.autograd.Function):
    """pooled = masked mean of weight[ids] over the sequence (ids > 0 are real tokens)."""

    @staticmethod
    def forward(ctx, weight, ids, padding_idx, scatter_mode, want_plan=False):
        require_gpu(weight, ids)
        if ids.dim() != 2:
            raise ValueError(f"ids must be (batch, seq_len), got shape {tuple(ids.shape)}")
        ids = ids.contiguous()
        ctx.plan = None
        plan_now = want_plan and scatter_mode == _lib.TT_SCATTER_SORTED
        # Where the sort forks onto its side stream (plan_fork_early): in a captured step, before
        # the gather, beside it, when the table fits the 256 MiB Infinity Cache (the gather then
        # reads the cache, and the latency-bound sort beside it costs it little: C3 0.8381 vs
        # 0.8419 ms/step), after it otherwise (an HBM-bound gather of a larger table: C5 1.8235
        # early vs 1.8178 after; profiles/r03p_c3_plan_fork_ab.txt, r03w_plan_fork_auto_ab.txt)
        # (round 4, same box: early 0.8256 vs late 0.8343 ms/step at C3, profiles/r04f_plan_fork_ab.txt);
        # in an eager step, after the gather (round 5, profiles/r05zl_plain_fork_ab.txt)
        early = plan_now and plan_fork_early(weight.numel() * weight.element_size())
        if early:
            deferred = getattr(weight, "_tt_deferred", None)
            group = deferred.gather_group if deferred is not None else None
            ctx.plan = BagPlan(ids, weight.shape[0], weight.shape[1], padding_idx, gather_group=group)
        pooled, denom = bag_mean_forward(weight, ids)
        if plan_now and not early:
            # forked after the gather: the sort runs beside the towers and the scorer (forked
            # before it, beside the gather, the step took 22 us longer: 0.887 vs 0.864 ms; again
            # after the weight-gradient fix, 0.8825 vs 0.8785: the gather holds the CUs and the
            # sort still ends beside the scorer -- both with the round-2 rocPRIM sort)
            deferred = getattr(weight, "_tt_deferred", None)
            group = deferred.gather_group if deferred is not None else None
            ctx.plan = BagPlan(ids, weight.shape[0], weight.shape[1], padding_idx, gather_group=group)
        ctx.save_for_backward(ids, denom)
        ctx.token = None
        if want_plan and scatter_mode == _lib.TT_SCATTER_SORTED:
            ctx.token = pooled._tt_bag_token = _BagGradToken(denom)
        ctx.V = weight.shape[0]
        ctx.padding_idx = padding_idx
        ctx.scatter_mode = scatter_mode
        ctx.weight_ref = weight
        return pooled

    @staticmethod
    def backward(ctx, d_pooled):
        ids, denom = ctx.saved_tensors
        weight = ctx.weight_ref
        plan, ctx.plan = ctx.plan, None
        tok, ctx.token = ctx.token, None
        if tok is not None and tok.grad is not None:
            # the sole consuming head already divided each row by its denominator
            if tok.grad.data_ptr() != d_pooled.data_ptr() or tok.grad.shape != d_pooled.shape:
                raise RuntimeError("bag output pre-scaled by its head was combined with another gradient")
            tok.grad = None
            denom = None
        if not ctx.needs_input_grad[0]:
            return None, None, None, None, None
        deferred = getattr(weight, "_tt_deferred", None)
        if deferred is not None:
            # A fused optimizer owns this table: hand it the factored gradient.
            deferred.parts.append((ids, d_pooled.contiguous(), denom, plan))
            deferred.added()
            return None, None, None, None, None
        if plan is not None:
            return bag_mean_backward_planned(d_pooled, denom, plan), None, None, None, None
        if denom is None:  # (no plan: an unplanned backward divides again; never taken by the head path)
            raise RuntimeError("pre-scaled bag gradient without a plan")
        grad = bag_mean_backward(d_pooled, denom, ids, ctx.V, ctx.padding_idx, ctx.scatter_mode)
        return grad, None, None, None, None


class ColumnPlan:
    """The sort plan of this rank's tokens (a BagPlan over the local ids, El wide) and, once
    ``exchange()`` ran, every rank's plan all-gathered on the plan's side stream: seg_all
    (world, V + 1) row starts and vals_all (world, nseq * L) sorted sequence indices, the inputs of
    tt_bag_col_reduce.  ``ready`` marks the exchange's end on the side stream."""

    __slots__ = ("plan", "seg_all", "vals_all", "nL", "ready")

    def __init__(self, ids: torch.Tensor, V: int, El: int, padding_idx):
        self.plan = BagPlan(ids, V, El, padding_idx)
        self.nL = self.plan.nseq * self.plan.L
        self.seg_all = self.vals_all = self.ready = None

    def exchange(self, col) -> None:
        """All-gather the plan's row starts and sorted indices (issued after the forward's pooled
        all-to-all, so the communicator does not hold that exchange behind the sort)."""
        from .distributed import all_gather_rows

        p = self.plan
        dev = p.buf.device
        offs = (ctypes.c_int64 * 3)()
        call("tt_bag_plan_layout", p.nseq, p.L, p.V, p.E, offs)
        base = (-p.buf.data_ptr()) % 256
        side = _lib.side_stream(dev)
        with torch.cuda.stream(side):  # behind the sort on its own stream
            vals = p.buf[base + offs[1]: base + offs[1] + 4 * self.nL].view(torch.int32)
            seg = p.buf[base + offs[2]: base + offs[2] + 4 * (p.V + 1)].view(torch.int32)
            self.vals_all = torch.empty(col.world * self.nL, dtype=torch.int32, device=dev)
            self.seg_all = torch.empty(col.world * (p.V + 1), dtype=torch.int32, device=dev)
            if self.nL:
                all_gather_rows(self.vals_all, vals, col.group)
            all_gather_rows(self.seg_all, seg, col.group)
            self.ready = torch.cuda.Event()
            self.ready.record(side)

    def wait(self) -> None:
        cur = torch.cuda.current_stream(self.plan.buf.device)
        cur.wait_event(self.ready)
        for t in (self.plan.buf, self.seg_all, self.vals_all):
            t.record_stream(cur)


def column_pooled_exchange(part: torch.Tensor, col, nseq: int) -> torch.Tensor:
    """part (world * nseq, El): this rank's columns of every rank's sequences (rank-major).  Returns
    this rank's (nseq, E) pooled rows: block s of the all-to-all is rank s's columns of them."""
    from .distributed import all_to_all_rows

    recv = torch.empty_like(part)
    all_to_all_rows(recv, part, col.group)
    return recv.view(col.world, nseq, col.El).permute(1, 0, 2).reshape(nseq, col.world * col.El)


def column_grad_exchange(gs: torch.Tensor, col) -> torch.Tensor:
    """gs (nseq, E): this rank's d_pooled / denom.  Returns (world * nseq, El): every rank's gs at this
    rank's columns, rank-major (block s of the all-to-all = rank s's sequences)."""
    from .distributed import all_to_all_rows

    nseq, W, El = gs.shape[0], col.world, col.El
    send = gs.view(nseq, W, El).permute(1, 0, 2).reshape(W * nseq, El)
    gs_all = torch.empty(W * nseq, El, dtype=gs.dtype, device=gs.device)
    all_to_all_rows(gs_all, send, col.group)
    return gs_all


class BagMeanPoolColumn(torch.autograd.Function):
    """BagMeanPool for a column-sharded table (distributed.ColumnTable, table_sync "column"):
    every rank's ids all-gathered, this rank's columns pooled for all of them from its slab
    (tt_bag_mean_fwd_cols, El wide, in the full-width sum order), the column blocks exchanged all-to-all, so each rank returns the
    whole pooled rows of its own sequences (encoders.py:62-72).  Backward: d_pooled / denom cut
    into column blocks and exchanged all-to-all; the factored gradient (every rank's gs at this
    rank's columns + the all-gathered plans) goes to the optimizer (tt_bag_col_reduce fused with
    AdamW on the slab)."""

    @staticmethod
    def forward(ctx, weight, ids, padding_idx, col, want_grad):
        from .distributed import all_gather_rows

        require_gpu(weight, ids)
        if ids.dim() != 2:
            raise ValueError(f"ids must be (batch, seq_len), got shape {tuple(ids.shape)}")
        ids = ids.contiguous()
        nseq, L = ids.shape
        W, El, V = col.world, col.El, col.V
        dev = weight.device
        cplan = ColumnPlan(ids, V, El, padding_idx) if want_grad else None  # local sort, side stream
        ids_all = ids.new_empty((W * nseq, L))
        all_gather_rows(ids_all, ids, col.group)
        part = torch.empty(W * nseq, El, dtype=_FLOAT, device=dev)
        den_all = torch.empty(W * nseq, dtype=_FLOAT, device=dev)
        if W * nseq:
            call("tt_bag_mean_fwd_cols", ptr(col.slab), V, El, weight.shape[1], ptr(ids_all),
                 _lib.ids_dtype_code(ids_all), W * nseq, L, L, ptr(part), ptr(den_all), stream_of(weight))
        pooled = column_pooled_exchange(part, col, nseq)
        denom = den_all[col.rank * nseq:(col.rank + 1) * nseq]
        if cplan is not None:
            cplan.exchange(col)
        ctx.cplan, ctx.col = cplan, col
        ctx.save_for_backward(denom)
        ctx.token = None
        if want_grad:
            ctx.token = pooled._tt_bag_token = _BagGradToken(denom)
        ctx.weight_ref = weight
        return pooled

    @staticmethod
    def backward(ctx, d_pooled):
        (denom,) = ctx.saved_tensors
        col, cplan = ctx.col, ctx.cplan
        ctx.cplan = None
        tok, ctx.token = ctx.token, None
        if not ctx.needs_input_grad[0] or cplan is None:
            return None, None, None, None, None
        if tok is not None and tok.grad is not None:
            if tok.grad.data_ptr() != d_pooled.data_ptr() or tok.grad.shape != d_pooled.shape:
                raise RuntimeError("bag output pre-scaled by its head was combined with another gradient")
            tok.grad = None
            gs = d_pooled.contiguous()  # the sole consuming head already divided by the denominators
        else:
            d_pooled = _contig_f32(d_pooled, "d_pooled")
            gs = torch.empty_like(d_pooled)
            call("tt_bag_scale_rows", ptr(d_pooled), ptr(denom), d_pooled.shape[0], d_pooled.shape[1], ptr(gs),
                 stream_of(d_pooled))
        nseq = gs.shape[0]
        gs_all = column_grad_exchange(gs, col)
        deferred = getattr(ctx.weight_ref, "_tt_deferred", None)
        if deferred is None:
            raise RuntimeError("a column-sharded table needs its optimizer (optim.AdamW(table_sync='column'))")
        deferred.parts.append(("column", gs_all, nseq, cplan))
        deferred.added()
        return None, None, None, None, None


def bag_col_update(col, parts, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor, adam_args: torch.Tensor) -> None:
    """The column-sharded table's AdamW step on its slab from the factored gradients of this step's
    bag calls (BagMeanPoolColumn): one fused launch for one call (tt_bag_col_reduce, grad NULL); for
    several calls on the table, their gradient rows are summed first, then one dense AdamW."""
    slab = col.slab

    def ws_for(cp):  # the hot-row path's scratch (pieces of rows longer than 128 merged tokens)
        n = _lib.lib().tt_bag_col_reduce_ws_size(col.V, col.world, cp.nL, col.El)
        return WORKSPACE.get("col_reduce", n, slab.device), n

    if len(parts) == 1:
        _, gs_all, nseq, cp = parts[0]
        cp.wait()
        ws, n = ws_for(cp)
        call("tt_bag_col_reduce_ex", ptr(cp.seg_all), ptr(cp.vals_all), cp.nL, col.world, nseq, ptr(gs_all), col.V,
             col.El, None, ptr(slab), ptr(exp_avg), ptr(exp_avg_sq), ptr(adam_args), ptr(ws), n, stream_of(slab))
    else:
        g = torch.zeros_like(slab)
        for _, gs_all, nseq, cp in parts:
            cp.wait()
            gi = torch.empty_like(slab)
            ws, n = ws_for(cp)
            call("tt_bag_col_reduce_ex", ptr(cp.seg_all), ptr(cp.vals_all), cp.nL, col.world, nseq, ptr(gs_all),
                 col.V, col.El, ptr(gi), None, None, None, None, ptr(ws), n, stream_of(slab))
            g += gi
        adamw_multi([(slab, g, exp_avg, exp_avg_sq, adam_args)])
    col.stale = True


def bag_mean_pool(weight: torch.Tensor, ids: torch.Tensor, padding_idx: int | None = 0,
                  scatter_mode: int = _lib.TT_SCATTER_SORTED) -> torch.Tensor:
    col = getattr(weight, "_tt_column", None)
    want_plan = torch.is_grad_enabled() and weight.requires_grad
    if col is not None and (want_plan or col.stale):  # data parallel, column-sharded table (ColumnTable):
        # collective.  A forward without gradient on a materialised table (after state_dict() or
        # materialize()) reads the full local weight instead: rank-local evaluation and search.
        return BagMeanPoolColumn.apply(weight, ids, padding_idx, col, want_plan)
    return BagMeanPool.apply(weight, ids, padding_idx, scatter_mode, want_plan)


# --------------------------------------------------------------------------------------------
# F.normalize(x, dim=-1), eps 1e-12   (twotower/encoders.py:77)
class L2Normalize(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        require_gpu(x)
        x = _contig_f32(x, "x")
        rows, H = x.shape
        out = torch.empty_like(x)
        norm = torch.empty(rows, dtype=_FLOAT, device=x.device)
        call("tt_l2norm_fwd", ptr(x), rows, H, ptr(out), ptr(norm), stream_of(x))
        ctx.save_for_backward(out, norm)
        return out

    @staticmethod
    def backward(ctx, dout):
        out, norm = ctx.saved_tensors
        dout = _contig_f32(dout, "dout")
        dx = torch.empty_like(out)
        call("tt_l2norm_bwd", ptr(dout), ptr(out), ptr(norm), out.shape[0], out.shape[1], ptr(dx), stream_of(out))
        return dx


def l2_normalize(x: torch.Tensor) -> torch.Tensor:
    return L2Normalize.apply(x)


class LayerNormL2Normalize(torch.autograd.Function):
    """F.normalize(layer_norm(x, gamma, beta, eps)) in one row pass each way (the AveragePooling
    projection tail, encoders.py:95-97,150); gamma/beta gradients by tt_colsum."""

    @staticmethod
    def forward(ctx, x, gamma, beta, eps):
        require_gpu(x, gamma, beta)
        x = _contig_f32(x, "x")
        rows, H = x.shape
        out = torch.empty_like(x)
        stats = torch.empty(rows, 3, dtype=_FLOAT, device=x.device)
        call("tt_ln_l2_fwd", ptr(x), rows, H, ptr(gamma), ptr(beta), float(eps), ptr(out), ptr(stats), stream_of(x))
        ctx.save_for_backward(x, gamma, beta, stats)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, gamma, beta, stats = ctx.saved_tensors
        dout = _contig_f32(dout, "dout")
        rows, H = x.shape
        dx = torch.empty_like(x)
        if H <= 1024 and H % 2 == 0:  # dgamma / dbeta folded per workgroup (tt_ln_l2_bwd_ex)
            dg, db = torch.empty(H, dtype=_FLOAT, device=x.device), torch.empty(H, dtype=_FLOAT, device=x.device)
            nbytes = _lib.lib().tt_ln_l2_bwd_ws_size(rows, H)
            ws = WORKSPACE.get("ln_l2_bwd", nbytes, x.device)
            call("tt_ln_l2_bwd_ex", ptr(dout), ptr(x), rows, H, ptr(gamma), ptr(beta), ptr(stats), ptr(dx), ptr(dg),
                 ptr(db), ptr(ws), ws.numel(), stream_of(x))
            return dx, dg, db, None
        gx, gb = torch.empty_like(x), torch.empty_like(x)
        call("tt_ln_l2_bwd", ptr(dout), ptr(x), rows, H, ptr(gamma), ptr(beta), ptr(stats), ptr(dx), ptr(gx),
             ptr(gb), stream_of(x))
        return dx, colsum(gx), colsum(gb), None


def layernorm_l2_normalize(x, gamma, beta, eps=1e-5):
    return LayerNormL2Normalize.apply(x, gamma, beta, eps)


# --------------------------------------------------------------------------------------------
# Tower feed-forward Linear(E,H) - ReLU - Linear(H,H)   (twotower/encoders.py:38-42)
def colsum(x: torch.Tensor) -> torch.Tensor:
    """x.sum(0) on the deterministic HIP column-sum (the nn.Linear bias gradient)."""
    require_gpu(x)
    x = _contig_f32(x, "x")
    rows, cols = x.shape
    if cols % 4:
        raise ValueError(f"colsum: hidden size {cols} must be a multiple of 4")
    out = torch.empty(cols, dtype=_FLOAT, device=x.device)
    nbytes = _lib.lib().tt_colsum_ws_size(rows, cols)
    ws = WORKSPACE.get("colsum", nbytes, x.device)
    call("tt_colsum", ptr(x), rows, cols, ptr(out), ptr(ws), ws.numel(), stream_of(x))
    return out


def _weight_grad(dy: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """dy^T x for tall N x H / N x E operands, K-split into S slabs (bmm) and summed: the
    library GEMM picks a 32x64 tile grid for the 256 x 256 output and leaves most CUs idle."""
    N = dy.shape[0]
    S = 1
    for cand in (16, 8, 4, 2):
        if N % cand == 0 and N // cand >= 1024:
            S = cand
            break
    if S == 1:
        return dy.t() @ x
    return torch.bmm(dy.view(S, N // S, -1).transpose(1, 2), x.view(S, N // S, -1)).sum(0)


class TowerFF(torch.autograd.Function):
    """y = relu(x W1^T + b1) W2^T + b2 with weight gradients on K-split GEMMs, bias gradients on
    tt_colsum and the ReLU mask fused into the backward product."""

    @staticmethod
    def forward(ctx, x, W1, b1, W2, b2):
        require_gpu(x)
        h = torch._addmm_activation(b1, x, W1.t())  # bias + ReLU in the hipBLASLt epilogue
        y = torch.addmm(b2, h, W2.t())
        ctx.save_for_backward(x, h, W1, W2)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, h, W1, W2 = ctx.saved_tensors
        dy = dy.contiguous()
        dh = dy @ W2
        call("tt_relu_bwd", ptr(dh), ptr(h), dh.numel(), stream_of(dh))
        dx = dh @ W1 if ctx.needs_input_grad[0] else None
        return dx, _weight_grad(dh, x), colsum(dh), _weight_grad(dy, h), colsum(dy)


def tower_ff(x, W1, b1, W2, b2):
    return TowerFF.apply(x, W1, b1, W2, b2)


HEAD_WIDTH = 256  # the width the scorer-side fusions (operand prep, fused L2 backward) are specialised for
HEAD_WIDTHS = (128, 256)  # H widths of the hand-written tower head (C2: 128; C3 / C5: 256)
EMB_WIDTHS = (64, 128, 256)  # its first Linear's input widths E (C1's char tower: E 64, H 128)


def _planes(W: torch.Tensor, transpose: bool) -> torch.Tensor:
    """The three bf16 planes of W (N x K), or of W^T (K x N) when transpose (tt_head_split's N, K are
    the planes' own rows and columns)."""
    N, K = W.shape if not transpose else (W.shape[1], W.shape[0])
    buf = torch.empty(_lib.lib().tt_head_planes_bytes(N, K), dtype=torch.uint8, device=W.device)
    call("tt_head_split", ptr(W.contiguous()), N, K, int(transpose), ptr(buf), stream_of(W))
    return buf


def _head_gemm(A: torch.Tensor, planes: torch.Tensor, epi: int, bias=None, mask=None, norms=None,
               N: int | None = None) -> torch.Tensor:
    """out (rows, N) = epi(A W^T) for the split planes of W (N x K); N defaults to K (square heads)."""
    rows, K = A.shape
    N = K if N is None else N
    out = torch.empty(rows, N, dtype=_FLOAT, device=A.device)
    nws = _lib.lib().tt_head_gemm_ws_size(rows, epi)
    ws = torch.empty(nws, dtype=torch.uint8, device=A.device) if nws else None
    call("tt_head_gemm", ptr(A), rows, A.stride(0), K, ptr(planes), N, epi, ptr(bias), ptr(mask), ptr(out),
         ptr(norms), ptr(ws), nws, stream_of(A))
    return out


_SCORER_PREP: list[tuple[int, int]] = []  # (query rows, compute dtype code) of an open scorer_prep()


def _prep_fusable(width: int, dt: int) -> bool:
    """tt_inbatch_l2_prep's shapes: H = 256 with bf16 operand copies (C3), H = 128 fp32 (C2)."""
    return (width == HEAD_WIDTH and dt != _lib.TT_F32) or (width == 128 and dt == _lib.TT_F32)


@contextlib.contextmanager
def scorer_prep(nq: int, compute_dtype: str):
    """While open, a TowerHead over rows [q (nq rows); candidates] also prepares the in-batch
    scorer's operands in its normalise pass (tt_inbatch_l2_prep): the bf16 copies and norms the
    loss would otherwise form in a pass of its own.  They ride on the head's output tensor
    (``_tt_inbatch_prep``) to InBatchSoftmaxLossPacked, which takes them once; any other consumer
    ignores them.  TwoTower opens it for its one-head fused forward when asked
    (``TwoTower.scorer_prep``, set by TrainStep for a bf16 in-batch loss)."""
    _SCORER_PREP.append((int(nq), _lib.compute_dtype_code(compute_dtype)))
    try:
        yield
    finally:
        _SCORER_PREP.pop()


class _L2Token:
    """Shared by a TowerHead whose output went to an in-batch loss under scorer_prep and that
    loss: under ``fused_head_backward`` the loss's backward applies the head's F.normalize
    backward in its combine (tt_inbatch_bwd_l2) and leaves dy here for the head."""

    __slots__ = ("norms", "dy")

    def __init__(self, norms: torch.Tensor):
        self.norms, self.dy = norms, None


_FUSED_HEAD_BWD = [0]  # > 0 while the caller runs a backward in which the head output feeds only the loss


@contextlib.contextmanager
def fused_head_backward():
    """Opened by train_step.TrainStep around its loss.backward(): the tower head's outputs reach
    the in-batch loss and nothing else, so the loss may hand the head the gradient after
    F.normalize (TT_FUSED_L2_BWD=0 turns it off)."""
    on = os.environ.get("TT_FUSED_L2_BWD", "1") != "0"
    _FUSED_HEAD_BWD[0] += on
    try:
        yield
    finally:
        _FUSED_HEAD_BWD[0] -= on


class TowerHead(torch.autograd.Function):
    """F.normalize(Linear(E,H)-ReLU-Linear(H,H)(x)) for H in {128, 256}, E in {64, 128, 256}
    (encoders.py:38-42,77) on the split-bf16 MFMA GEMMs with fused epilogues: bias + ReLU (+ the
    ReLU bitmask), bias + row L2 normalise (forward); the ReLU mask fused into dh = dy W2, dx = dh W1
    (backward).  Weight and bias gradients on the split-bf16 MFMA kernels (tt_head_wgrad2 in one
    launch for E = H, tt_head_wgrad_ex per Linear otherwise)."""

    @staticmethod
    def forward(ctx, x, W1, b1, W2, b2):
        require_gpu(x, W1, W2)
        ctx.bag_token = x._tt_bag_token if _SOLE_HEAD and _SOLE_HEAD[-1] is x else None
        x = _contig_f32(x, "x")
        rows, E = x.shape
        H = W1.shape[0]  # width = H (HEAD_WIDTHS), E in EMB_WIDTHS
        width = H
        n1, n2 = _head_planes_bytes(E, H)
        planes = _PLANES_DONE.pop((W1.data_ptr(), W2.data_ptr()), None)  # formed by the gather (same stream)
        if planes is None or planes.numel() != 2 * (n1 + n2):
            planes = torch.empty(2 * (n1 + n2), dtype=torch.uint8, device=x.device)  # W1, W2, W1^T, W2^T
            call("tt_head_split_ff2", ptr(_contig_f32(W1, "W1")), ptr(_contig_f32(W2, "W2")), E, H, ptr(planes),
                 stream_of(x))
        p_w1, p_w2 = planes[:n1], planes[n1:n1 + n2]
        norm = torch.empty(rows, dtype=_FLOAT, device=x.device)
        req = _SCORER_PREP[-1] if _SCORER_PREP and _prep_fusable(width, _SCORER_PREP[-1][1]) else None
        prep = req is not None and 0 < req[0] < rows
        mask = torch.empty(_lib.lib().tt_head_relu_mask_bytes(rows) // 4, dtype=torch.int32, device=x.device)
        h = _head_gemm(x, p_w1, 0, bias=b1, mask=mask, N=H)
        out = _head_gemm(h, p_w2, 4, bias=b2) if prep else _head_gemm(h, p_w2, 1, bias=b2, norms=norm)
        if prep:
            nq, dt = req  # normalise pass fused with the in-batch scorer's operand prep
            ws = torch.empty(_lib.lib().tt_inbatch_ws_size(nq, rows - nq, width, dt), dtype=torch.uint8,
                             device=x.device)
            call("tt_inbatch_l2_prep", ptr(out), nq, rows - nq, width, dt, ptr(norm), ptr(ws), ws.numel(),
                 stream_of(x))
            ctx.l2_token = _L2Token(norm)
            out._tt_inbatch_prep = (nq, rows - nq, dt, ws, ctx.l2_token)
        if req is None or not 0 < req[0] < rows:
            # a loss that takes the whole output as one tensor (MultiNegLossPacked) may apply
            # F.normalize's backward itself under fused_head_backward and leave dy here
            ctx.l2_token = _L2Token(norm)
            out._tt_l2_token = ctx.l2_token
        ctx.save_for_backward(x, h, mask, out, norm, planes)
        sides = {id(getattr(w, "_tt_side_grads", None)) for w in (W1, b1, W2, b2)}
        ctx.side_grads = W1._tt_side_grads if len(sides) == 1 and hasattr(W1, "_tt_side_grads") else None
        ctx.params = (W1, b1, W2, b2) if ctx.side_grads is not None else None
        if ctx.side_grads is not None and ctx.side_grads.active:
            for w in ctx.params:
                ctx.side_grads.use(w)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, h, mask, out, norm, planes = ctx.saved_tensors
        E, H = x.shape[1], out.shape[1]
        n1, n2 = _lib.lib().tt_head_planes_bytes(H, E), _lib.lib().tt_head_planes_bytes(H, H)
        p_w1t, p_w2t = planes[n1 + n2:2 * n1 + n2], planes[2 * n1 + n2:]
        tok, ctx.l2_token = ctx.l2_token, None
        if tok is not None and tok.dy is not None:  # the loss applied F.normalize's backward (tt_inbatch_bwd_l2)
            if tok.dy.data_ptr() != dout.data_ptr() or tok.dy.shape != dout.shape:
                raise RuntimeError("tower head output fed the fused in-batch loss and another consumer")
            dy, tok.dy = tok.dy, None
        else:
            dout = _contig_f32(dout, "dout")
            dy = torch.empty_like(out)
            call("tt_l2norm_bwd", ptr(dout), ptr(out), ptr(norm), out.shape[0], out.shape[1], ptr(dy),
                 stream_of(out))
        side = ctx.side_grads
        N = H
        dW1, dW2 = torch.empty(H, E, dtype=_FLOAT, device=dy.device), torch.empty(H, H, dtype=_FLOAT, device=dy.device)
        db1, db2 = (torch.empty(H, dtype=_FLOAT, device=dy.device) for _ in range(2))
        # The optimizer joins these (optim.AdamW), so the weight gradients may run on a side stream
        # beside what follows on this one: dx feeds the fused table scatter + AdamW, an
        # HBM-bound pass the MFMA-bound weight-gradient kernels overlap.  Autograd must hand the
        # returned buffers to .grad as they are (checked at the join): no extra references.
        on_side = not (side is None or not side.active or not all(ctx.needs_input_grad[1:5])
                       or not side.single_use(ctx.params)
                       or any(p.grad is not None for p in ctx.params))  # (an existing .grad accumulates now)
        main = torch.cuda.current_stream(dy.device)
        aux = _lib.side_stream(dy.device, "wgrad") if on_side else None

        def wgrad_aside(G, X, dW, db):
            aux.wait_stream(main)
            # cross-stream lifetimes (also during capture, where the allocator then defers the
            # blocks' reuse to the end of the capture instead of handing them to a later node)
            for t in (G, X, dW, db):
                t.record_stream(aux)
            with torch.cuda.stream(aux):
                head_wgrad(G, X, dW, db)

        tok, ctx.bag_token = ctx.bag_token, None
        dx = None
        dh = _head_gemm(dy, p_w2t, 2, mask=mask, N=H)
        if ctx.needs_input_grad[0] and tok is not None:  # dx / denom for the bag backward (epi 5)
            dx = _head_gemm(dh, p_w1t, 5, bias=tok.denom, N=E)
            tok.grad = dx
        elif ctx.needs_input_grad[0]:
            dx = _head_gemm(dh, p_w1t, 3, N=E)
        two = E == H  # square heads: both weight gradients in one launch (tt_head_wgrad2)
        if not on_side:
            if two:
                head_wgrad2_reduce(head_wgrad2(dh, x, dy, h), dW1, db1, dW2, db2)
            else:
                head_wgrad(dh, x, dW1, db1)
                head_wgrad(dy, h, dW2, db2)
            return dx, dW1, db1, dW2, db2
        # forked after the dx GEMM: forked earlier (dW2 beside the dh GEMM, dW1 beside the dx GEMM)
        # they time-share the CUs with those GEMMs and the step took 20 us longer.  Both weight
        # gradients are ONE launch (tt_head_wgrad2), whose slab partials the optimizer's join sums
        # on its own stream: a chain of four side-stream kernels starved behind the table reduce,
        # which holds every CU once it runs (its last kernels ran 10-30x their own time).
        if two:
            ws = torch.empty(_lib.lib().tt_head_wgrad2_ws_size(dy.shape[0], N), dtype=torch.uint8, device=dy.device)
            aux.wait_stream(main)  # dh, dy written on this stream
            ws.record_stream(aux)
            for t in (dh, dy, x, h):
                t.record_stream(aux)
            with torch.cuda.stream(aux):
                head_wgrad2(dh, x, dy, h, ws)
            done = torch.cuda.Event()
            done.record(aux)
            side.add(done, zip(ctx.params, (dW1, db1, dW2, db2)), finalize=_Wgrad2Sums(ws, ctx.params))
            return dx, dW1, db1, dW2, db2
        wgrad_aside(dh, x, dW1, db1)
        wgrad_aside(dy, h, dW2, db2)
        done = torch.cuda.Event()
        done.record(aux)
        side.add(done, zip(ctx.params, (dW1, db1, dW2, db2)))
        return dx, dW1, db1, dW2, db2


def head_wgrad(G: torch.Tensor, X: torch.Tensor, dW: torch.Tensor | None = None,
               db: torch.Tensor | None = None) -> tuple[torch.Tensor, torch.Tensor]:
    """(G^T X, G.sum(0)) for fp32 G (rows, NG), X (rows, NX) on the split-bf16 MFMA kernel
    (tt_head_wgrad_ex: NG in {128, 256}, NX in {64, 128, 256})."""
    rows, NG = G.shape
    NX = X.shape[1]
    dW = torch.empty(NG, NX, dtype=_FLOAT, device=G.device) if dW is None else dW
    db = torch.empty(NG, dtype=_FLOAT, device=G.device) if db is None else db
    nws = _lib.lib().tt_head_wgrad_ex_ws_size(rows, NG, NX)
    ws = torch.empty(nws, dtype=torch.uint8, device=G.device)
    call("tt_head_wgrad_ex", ptr(G), ptr(X), rows, NG, NX, ptr(dW), ptr(db), ptr(ws), nws, stream_of(G))
    return dW, db


def head_wgrad2(G1: torch.Tensor, X1: torch.Tensor, G2: torch.Tensor, X2: torch.Tensor,
                ws: torch.Tensor | None = None) -> torch.Tensor:
    """Slab partials of both head weight gradients in one launch (tt_head_wgrad2); returns ws."""
    rows, N = G1.shape
    nbytes = _lib.lib().tt_head_wgrad2_ws_size(rows, N)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=G1.device) if ws is None else ws
    call("tt_head_wgrad2", ptr(G1), ptr(X1), ptr(G2), ptr(X2), rows, N, ptr(ws), ws.numel(),
         torch.cuda.current_stream(G1.device).cuda_stream)
    return ws


class _Wgrad2Sums:
    """The join's finalize for tt_head_wgrad2's partials: called, it queues the fixed-order slab
    sums (tt_head_wgrad2_reduce) on the joining stream (the optimizer's, or the DP all-reduce's)
    into the .grad tensors autograd stole from the backward (no reference to them is kept here:
    an extra one would make autograd copy instead).  An optimizer that forms the sums inside its
    own update launch (optim.AdamW, tt_adamw_multi_ex) takes ``grad_parts()`` instead."""

    def __init__(self, ws: torch.Tensor, params):
        self.ws, self.params = ws, tuple(params)

    def __call__(self) -> None:
        self.ws.record_stream(torch.cuda.current_stream(self.ws.device))
        head_wgrad2_reduce(self.ws, *(p.grad for p in self.params))

    def grad_parts(self) -> dict:
        self.ws.record_stream(torch.cuda.current_stream(self.ws.device))
        N = self.params[0].shape[0]
        out = {}
        for k, p in enumerate(self.params):
            off, stride = ctypes.c_int64(), ctypes.c_int64()
            slabs = _lib.lib().tt_head_wgrad2_parts(N, k, ctypes.byref(off), ctypes.byref(stride))
            if slabs < 0:
                raise RuntimeError(_lib.lib().tt_last_error().decode())
            out[id(p)] = (ptr(self.ws) + 4 * off.value, stride.value, slabs, self.ws)
        return out


def head_wgrad2_reduce(ws: torch.Tensor, dW1, db1, dW2, db2) -> None:
    """(G1^T X1, colsum G1, G2^T X2, colsum G2) from tt_head_wgrad2's partials, on the current stream."""
    call("tt_head_wgrad2_reduce", ptr(ws), dW1.shape[0], ptr(dW1), ptr(db1), ptr(dW2), ptr(db2),
         torch.cuda.current_stream(ws.device).cuda_stream)


def tower_head(x, W1, b1, W2, b2):
    return TowerHead.apply(x, W1, b1, W2, b2)


def linear_widths_ok(E: int, H: int) -> bool:
    """(in E, out H) shapes of the hand-written Linear (LinearHead): tt_head_gemm epi 4 forward
    (K = E, N = H), epi 3 dx (K = H, N = E), tt_head_wgrad_ex (NG = H, NX = E)."""
    return E in EMB_WIDTHS and H in HEAD_WIDTHS


class LinearHead(torch.autograd.Function):
    """y = x W^T + b on the split-bf16 MFMA head kernels (fp32 accuracy): AveragePoolingTower's
    projection Linear(E, H) (encoders.py:84-155), forward tt_head_gemm epi 4 (bias), backward dx by
    epi 3 on the planes of W^T, dW and db by tt_head_wgrad_ex."""

    @staticmethod
    def forward(ctx, x, W, b):
        require_gpu(x, W, b)
        x = _contig_f32(x, "x")
        H, E = W.shape
        y = _head_gemm(x, _planes(_contig_f32(W, "W"), False), 4, bias=_contig_f32(b, "b"), N=H)
        ctx.save_for_backward(x, W)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, W = ctx.saved_tensors
        dy = _contig_f32(dy, "dy")
        dx = _head_gemm(dy, _planes(W, True), 3, N=W.shape[1]) if ctx.needs_input_grad[0] else None
        dW, db = head_wgrad(dy, x)
        return dx, dW, db


def linear(x, W, b):
    return LinearHead.apply(x, W, b)


# --------------------------------------------------------------------------------------------
# contrastive_triplet_loss   (twotower/losses.py:9-44)
def _triplet_fwd(q, p, n, margin):
    B, H = q.shape
    rows = torch.empty(B, dtype=_FLOAT, device=q.device)
    loss = torch.empty((), dtype=_FLOAT, device=q.device)
    call("tt_triplet_fwd", ptr(q), ptr(p), ptr(n), B, H, float(margin), ptr(rows), ptr(loss), stream_of(q))
    return loss


def _triplet_bwd(q, p, n, margin, g, dq, dp, dn):
    B, H = q.shape
    g = g.to(_FLOAT).contiguous().reshape(1)
    call("tt_triplet_bwd", ptr(q), ptr(p), ptr(n), B, H, margin, ptr(g), ptr(dq), ptr(dp), ptr(dn), stream_of(q))


class TripletLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, p, n, margin):
        require_gpu(q, p, n)
        q, p, n = (_contig_f32(t, nm) for t, nm in ((q, "q"), (p, "p"), (n, "n")))
        ctx.save_for_backward(q, p, n)
        ctx.margin = float(margin)
        return _triplet_fwd(q, p, n, margin)

    @staticmethod
    def backward(ctx, g):
        q, p, n = ctx.saved_tensors
        dq, dp, dn = torch.empty_like(q), torch.empty_like(p), torch.empty_like(n)
        _triplet_bwd(q, p, n, ctx.margin, g, dq, dp, dn)
        return dq, dp, dn, None


class TripletLossPacked(torch.autograd.Function):
    """Same loss on one (3B, H) tensor holding [q; p; n] (TwoTower's fused output): the gradient
    is written as one tensor, so autograd never runs the split backward (zeros + cat)."""

    @staticmethod
    def forward(ctx, qpn, margin):
        require_gpu(qpn)
        qpn = _contig_f32(qpn, "qpn")
        q, p, n = torch.chunk(qpn, 3)
        ctx.save_for_backward(qpn)
        ctx.margin = float(margin)
        return _triplet_fwd(q, p, n, margin)

    @staticmethod
    def backward(ctx, g):
        (qpn,) = ctx.saved_tensors
        grad = torch.empty_like(qpn)
        _triplet_bwd(*torch.chunk(qpn, 3), ctx.margin, g, *torch.chunk(grad, 3))
        return grad, None


# --------------------------------------------------------------------------------------------
# multiple_negatives_loss   (twotower/losses.py:47-85)
class MultiNegLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, p, negs, inv_tau):
        require_gpu(q, p, negs)
        q, p, negs = _contig_f32(q, "q"), _contig_f32(p, "p"), _contig_f32(negs, "negs")
        B, H = q.shape
        N = negs.shape[1]
        rows = torch.empty(B, dtype=_FLOAT, device=q.device)
        loss = torch.empty((), dtype=_FLOAT, device=q.device)
        call("tt_multi_neg_fwd", ptr(q), ptr(p), ptr(negs), B, N, H, float(inv_tau), ptr(rows), ptr(loss),
             stream_of(q))
        ctx.save_for_backward(q, p, negs)
        ctx.inv_tau = float(inv_tau)
        return loss

    @staticmethod
    def backward(ctx, g):
        q, p, negs = ctx.saved_tensors
        B, H = q.shape
        N = negs.shape[1]
        g = g.to(_FLOAT).contiguous().reshape(1)
        dq, dp, dnegs = torch.empty_like(q), torch.empty_like(p), torch.empty_like(negs)
        call("tt_multi_neg_bwd", ptr(q), ptr(p), ptr(negs), B, N, H, ctx.inv_tau, ptr(g), ptr(dq), ptr(dp),
             ptr(dnegs), stream_of(q))
        return dq, dp, dnegs, None


class MultiNegLossPacked(torch.autograd.Function):
    """The same loss on one ((2 + K) B, H) tensor [q; p; negatives (B K rows, query-major)]
    (TwoTower's fused output): the three gradients are written into one tensor, so autograd
    runs no split backward (a cat of the three, 50 MB at C5, on the step's critical path)."""

    @staticmethod
    def forward(ctx, qpn, B, K, inv_tau):
        require_gpu(qpn)
        qpn = _contig_f32(qpn, "qpn")
        H = qpn.shape[1]
        if qpn.shape[0] != (2 + K) * B:
            raise ValueError(f"packed multiple-negatives input must have (2 + K) B = {(2 + K) * B} rows")
        rows = torch.empty(B, dtype=_FLOAT, device=qpn.device)
        loss = torch.empty((), dtype=_FLOAT, device=qpn.device)
        q, p, n = qpn[:B], qpn[B:2 * B], qpn[2 * B:]
        call("tt_multi_neg_fwd", ptr(q), ptr(p), ptr(n), B, K, H, float(inv_tau), ptr(rows), ptr(loss), stream_of(qpn))
        ctx.save_for_backward(qpn)
        ctx.meta = (B, K, float(inv_tau))
        tok = getattr(qpn, "_tt_l2_token", None)  # the tower head's output itself, whole
        ctx.l2_token = tok if tok is not None and tok.norms.shape[0] == qpn.shape[0] and H == 256 and K <= 15 else None
        return loss

    @staticmethod
    def backward(ctx, g):
        (qpn,) = ctx.saved_tensors
        B, K, inv_tau = ctx.meta
        H = qpn.shape[1]
        g = g.to(_FLOAT).contiguous().reshape(1)
        grad = torch.empty_like(qpn)
        tok, ctx.l2_token = ctx.l2_token, None
        if tok is not None and _FUSED_HEAD_BWD[0] > 0:  # the head's F.normalize backward in the same pass
            call("tt_multi_neg_bwd_l2", ptr(qpn), B, K, ptr(tok.norms), inv_tau, ptr(g), ptr(grad), stream_of(qpn))
            tok.dy = grad
            return grad, None, None, None
        q, p, n = qpn[:B], qpn[B:2 * B], qpn[2 * B:]
        call("tt_multi_neg_bwd", ptr(q), ptr(p), ptr(n), B, K, H, inv_tau, ptr(g), ptr(grad[:B]), ptr(grad[B:2 * B]),
             ptr(grad[2 * B:]), stream_of(qpn))
        return grad, None, None, None


# --------------------------------------------------------------------------------------------
# in_batch_sampled_softmax_loss   (twotower/losses.py:88-118), fused MFMA scorer
_BWD_FORMS = {"recompute": _lib.TT_INBATCH_BWD_RECOMPUTE, "stored": _lib.TT_INBATCH_BWD_STORED}


def set_inbatch_backward(form: str) -> str:
    """Select the single-process bf16 / fp32 in-batch backward process-wide ("stored": G from the
    forward's stored probabilities, bf16 or fp32 as the scorer computes, the default; "recompute":
    recompute S = Q D^T) and return the previous form.  Switch only between steps, never between a
    forward and its backward."""
    prev = _lib.lib().tt_inbatch_set_backward(_BWD_FORMS[form])
    return {v: k for k, v in _BWD_FORMS.items()}[prev]


def get_inbatch_backward() -> str:
    """The current single-process bf16 / fp32 in-batch backward form ("stored" or "recompute")."""
    return {v: k for k, v in _BWD_FORMS.items()}[_lib.lib().tt_inbatch_set_backward(-1)]


def _inbatch_fwd(ctx, q, d, inv_tau, label_off, compute_dtype, grad_scale, want_grad, prep=None, defer_mean=False):
    B, H = q.shape
    M = d.shape[0]
    if d.shape[1] != H:
        raise ValueError(f"q is (B, {H}) but d is {tuple(d.shape)}")
    dt = _lib.compute_dtype_code(compute_dtype)
    dev = q.device
    nbytes = _lib.lib().tt_inbatch_ws_size(B, M, H, dt)
    if prep is not None and prep[:3] == (B, M, dt) and prep[3].numel() >= nbytes:
        ws, entry = prep[3], "tt_inbatch_fwd_prepped"  # operands prepared by the head's normalise pass
    else:
        ws, entry = torch.empty(nbytes, dtype=torch.uint8, device=dev), "tt_inbatch_fwd"
    # ws carries the bf16 operands to backward
    lse = torch.empty(B, dtype=_FLOAT, device=dev)
    rows = torch.empty(B, dtype=_FLOAT, device=dev)
    loss = torch.empty((), dtype=_FLOAT, device=dev)
    dqu = torch.empty(B, H, dtype=_FLOAT, device=dev) if want_grad else None
    call(entry, ptr(q), ptr(d), B, M, H, dt, float(inv_tau), int(label_off), int(want_grad),
         ptr(lse), ptr(rows), None if defer_mean else ptr(loss), ptr(dqu), ptr(ws), ws.numel(), stream_of(q))
    ctx.meta = (B, M, H, dt, float(inv_tau), int(label_off), float(1.0 / B) if grad_scale is None else float(grad_scale))
    ctx.deferred_mean = (rows, loss) if defer_mean else None
    return loss, lse, dqu, ws


def _inbatch_bwd(meta, q, d, lse, dqu, ws, g, dq, dd, mean=None):
    """mean = (loss_rows, loss): the forward deferred the loss mean; the combine launch forms it."""
    B, M, H, dt, inv_tau, label_off, grad_scale = meta
    g = g.to(_FLOAT).contiguous().reshape(1)
    call("tt_inbatch_bwd", ptr(q), ptr(d), B, M, H, dt, inv_tau, label_off, ptr(lse), ptr(dqu), ptr(g), grad_scale,
         ptr(dq), ptr(dd), ptr(mean[0]) if mean else None, ptr(mean[1]) if mean else None, ptr(ws), ws.numel(),
         stream_of(q))


class InBatchSoftmaxLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, d, inv_tau, label_off, compute_dtype, grad_scale):
        require_gpu(q, d)
        q, d = _contig_f32(q, "q"), _contig_f32(d, "d")
        want_grad = bool(ctx.needs_input_grad[0] or ctx.needs_input_grad[1])
        loss, lse, dqu, ws = _inbatch_fwd(ctx, q, d, inv_tau, label_off, compute_dtype, grad_scale, want_grad)
        if want_grad:
            ctx.save_for_backward(q, d, lse, dqu, ws)
        return loss

    @staticmethod
    def backward(ctx, g):
        q, d, lse, dqu, ws = ctx.saved_tensors
        dq, dd = torch.empty_like(q), torch.empty_like(d)
        _inbatch_bwd(ctx.meta, q, d, lse, dqu, ws, g, dq, dd)
        return dq, dd, None, None, None, None


class InBatchSoftmaxLossPacked(torch.autograd.Function):
    """In-batch loss on one (B + M, H) tensor [q; candidates] (TwoTower's fused output): dq and
    dd are written into one gradient tensor (no split backward)."""

    @staticmethod
    def forward(ctx, qd, nq, inv_tau, compute_dtype, grad_scale):
        require_gpu(qd)
        prep = qd.__dict__.pop("_tt_inbatch_prep", None)  # taken once (TowerHead under scorer_prep)
        qd = _contig_f32(qd, "qd")
        q, d = qd[:nq], qd[nq:]
        want_grad = bool(ctx.needs_input_grad[0])
        ctx.l2_token = prep[4] if prep is not None else None
        # inside TrainStep (deferred_loss_mean) the loss is read only after the step: its mean is
        # formed by the backward's combine launch (tt_inbatch_bwd_l2, or tt_inbatch_bwd when the head's L2
        # backward is not fused) instead of a launch of its own
        # between the forward combine and the backward engine
        defer = want_grad and _DEFER_MEAN[0] > 0 and os.environ.get("TT_DEFER_MEAN", "1") != "0"
        loss, lse, dqu, ws = _inbatch_fwd(ctx, q, d, inv_tau, 0, compute_dtype, grad_scale, want_grad,
                                          prep[:4] if prep is not None else None, defer_mean=defer)
        if want_grad:
            ctx.save_for_backward(qd, lse, dqu, ws)
        ctx.nq = nq
        return loss

    @staticmethod
    def backward(ctx, g):
        qd, lse, dqu, ws = ctx.saved_tensors
        grad = torch.empty_like(qd)
        nq = ctx.nq
        tok, ctx.l2_token = ctx.l2_token, None
        B, M, H, dt, inv_tau, label_off, grad_scale = ctx.meta
        dm, ctx.deferred_mean = ctx.deferred_mean, None
        if tok is not None and _FUSED_HEAD_BWD[0] > 0 and _l2_fusable(H, dt):
            # the head's F.normalize backward in the combine: grad is the head's dy (see _L2Token)
            gs = g.to(_FLOAT).contiguous().reshape(1)
            call("tt_inbatch_bwd_l2", ptr(qd), B, M, H, dt, inv_tau, label_off, ptr(lse), ptr(dqu), ptr(gs),
                 grad_scale, ptr(tok.norms), ptr(grad), ptr(dm[0]) if dm else None, ptr(dm[1]) if dm else None,
                 ptr(ws), ws.numel(), stream_of(qd))
            tok.dy = grad
            return grad, None, None, None, None
        _inbatch_bwd(ctx.meta, qd[:nq], qd[nq:], lse, dqu, ws, g, grad[:nq], grad[nq:], mean=dm)
        return grad, None, None, None, None


def _l2_fusable(H: int, dt: int) -> bool:
    """tt_inbatch_bwd_l2's shapes: H = 256 with bf16 operands (C3), H = 128 fp32 (C2)."""
    return (H == HEAD_WIDTH and dt != _lib.TT_F32) or (H == 128 and dt == _lib.TT_F32)


_DEFER_MEAN = [0]  # > 0 while a caller (TrainStep) runs the backward before anyone reads the loss


@contextlib.contextmanager
def deferred_loss_mean():
    """Declare that the loss of the forward run inside is read only after its backward has run
    (TrainStep): the in-batch loss may then leave its mean to the backward's combine launch."""
    _DEFER_MEAN[0] += 1
    try:
        yield
    finally:
        _DEFER_MEAN[0] -= 1


_UNIFORM_SEED = [0]  # > 0 while a caller guarantees every rank seeds its loss backward alike


@contextlib.contextmanager
def uniform_loss_seed():
    """Declare that every data-parallel rank seeds this backward with the same d(loss) (TrainStep:
    1/world), so InBatchSoftmaxLossOwned skips the seed exchange.  A module-level count, not a
    thread-local: autograd runs GPU backward functions on its own device threads."""
    _UNIFORM_SEED[0] += 1
    try:
        yield
    finally:
        _UNIFORM_SEED[0] -= 1


def _rank_seeds(lse2_all: torch.Tensor, g: torch.Tensor, B: int, world: int, group):
    """Per-rank backward seeds for the candidate-owner backward: every rank's seed is gathered
    and the reference seed g_ref = max_r g_r is what the kernel applies, with rank r's query
    terms weighed by g_r / g_ref through their lse2 (the kernel forms 2^(x c2 - lse2_i), so
    lse2_i -= log2(g_r / g_ref); a rank seeded 0 contributes nothing: lse2 = +inf).  The caller
    rescales this rank's dq by g / g_ref and moves its label terms from g_ref to g.  Equal seeds
    give shifts and corrections of exactly 0 (the same bits as without the exchange).  Negative
    seeds cannot be folded and fail loudly (device assert).  -> (lse2_all, g_ref)"""
    from .distributed import all_gather_rows

    g_all = torch.empty(world, dtype=_FLOAT, device=g.device)
    all_gather_rows(g_all, g.reshape(1), group)
    torch._assert_async((g_all >= 0).all(), "in-batch loss: data-parallel backward seeds must be >= 0")
    g_ref = g_all.max().reshape(1)
    ratio = g_all / torch.where(g_ref > 0, g_ref, torch.ones_like(g_ref))
    shift = torch.where(ratio > 0, torch.log2(ratio), torch.full_like(ratio, float("-inf")))
    out = lse2_all.clone()
    out[:world * B] -= shift.repeat_interleave(B)
    return out, g_ref


class InBatchSoftmaxLossOwned(torch.autograd.Function):
    """Data-parallel in-batch loss with cross-device negatives and candidate-owner gradients
    (bf16 / bf16_split).  Forward: every rank's bf16 candidate copies and norm maxima are
    all-gathered (half the bytes of fp32 rows) and this rank's queries are scored against all
    of them.  The bf16 query copies and lse2 are all-gathered asynchronously (overlapping the
    forward scorer); the backward computes the gradient of this rank's OWN candidates over every
    rank's queries, so no candidate gradient is reduce-scattered.  Every rank's loss must be
    seeded alike (TrainStep: 1/world, declared by ops.uniform_loss_seed()); otherwise the ranks'
    seeds are all-gathered in the backward and each remote query's terms take its own rank's seed
    (_rank_seeds)."""

    @staticmethod
    def forward(ctx, q, d, inv_tau, compute_dtype, grad_scale, group):
        from .distributed import all_gather_rows

        require_gpu(q, d)
        q, d = _contig_f32(q, "q"), _contig_f32(d, "d")
        B, H = q.shape
        M = d.shape[0]
        if d.shape[1] != H:
            raise ValueError(f"q is (B, {H}) but d is {tuple(d.shape)}")
        dt = _lib.compute_dtype_code(compute_dtype)
        if dt == _lib.TT_F32:
            raise ValueError("candidate-owner gradients need a bf16 compute dtype")
        world, rank = torch.distributed.get_world_size(group), torch.distributed.get_rank(group)
        dev, T, P = q.device, _lib.TT_INBATCH_TAIL_ROWS, _lib.TT_INBATCH_MAX_PARTS
        st = stream_of(q)
        bf = torch.bfloat16
        qb = torch.empty(B + T, H, dtype=bf, device=dev)
        qnorm = torch.empty(B, dtype=_FLOAT, device=dev)
        call("tt_inbatch_prep_rows", ptr(q), B, H, ptr(qb), ptr(qnorm), None, st)
        db = torch.empty(M + T, H, dtype=bf, device=dev)
        parts = torch.empty(P, dtype=_FLOAT, device=dev)
        call("tt_inbatch_prep_rows", ptr(d), M, H, ptr(db), None, ptr(parts), st)
        # bf16 rows travel as bytes (any backend), rank-major; the zero tail stays local.  From 4
        # ranks on (M a multiple of 64) the forward runs in two launches: this rank's own
        # candidates are scored while the other ranks' rows arrive.  Splitting costs 35-39 us on
        # one GPU (tools/mb.py split_fwd: the local launch leaves CUs to the collective); the
        # gather it hides grows with N (~0.1 ms at 4 ranks).  TT_INBATCH_OVERLAP=1 / 0 forces it.
        ov = os.environ.get("TT_INBATCH_OVERLAP", "auto")
        split = M % 64 == 0 and (ov == "1" or (ov == "auto" and world >= 4))
        db_all = torch.empty(world * M + T, H, dtype=bf, device=dev)
        db_all[world * M:].zero_()
        parts_all = torch.empty(world * P, dtype=_FLOAT, device=dev)
        w_p = all_gather_rows(parts_all, parts, group, async_op=split)
        w_d = all_gather_rows(db_all[:world * M].view(torch.uint8), db[:M].view(torch.uint8), group, async_op=split)
        qb_all = torch.empty(world * B + T, H, dtype=bf, device=dev)
        qb_all[world * B:].zero_()
        w_q = all_gather_rows(qb_all[:world * B].view(torch.uint8), qb[:B].view(torch.uint8), group, async_op=True)
        want_grad = bool(ctx.needs_input_grad[0] or ctx.needs_input_grad[1])
        ws = torch.empty(_lib.lib().tt_inbatch_ex_ws_size(B, world * M, world * B, M, H, dt), dtype=torch.uint8,
                         device=dev)
        lse = torch.empty(B, dtype=_FLOAT, device=dev)
        lse2 = torch.empty(B, dtype=_FLOAT, device=dev)
        rows = torch.empty(B, dtype=_FLOAT, device=dev)
        loss = torch.empty((), dtype=_FLOAT, device=dev)
        dqu = torch.empty(B, H, dtype=_FLOAT, device=dev) if want_grad else None
        if split:
            call("tt_inbatch_fwd_ex_local", ptr(qb), ptr(qnorm), B, ptr(db), ptr(parts), P, M, world * M, rank * M,
                 H, dt, float(inv_tau), ptr(ws), ws.numel(), st)
            w_p.wait()
            w_d.wait()
            call("tt_inbatch_fwd_ex_remote", ptr(qb), ptr(qnorm), B, ptr(db_all), ptr(parts_all), world * P,
                 ptr(parts), P, M, world * M, rank * M, H, dt, float(inv_tau), int(want_grad), ptr(lse), ptr(lse2),
                 ptr(rows), ptr(loss), ptr(dqu), ptr(ws), ws.numel(), st)
        else:
            call("tt_inbatch_fwd_ex", ptr(qb), ptr(qnorm), B, ptr(db_all), ptr(parts_all), world * P, world * M, H,
                 dt, float(inv_tau), rank * M, int(want_grad), ptr(lse), ptr(lse2), ptr(rows), ptr(loss), ptr(dqu),
                 ptr(ws), ws.numel(), st)
        lse2_all = torch.empty(world * B + T, dtype=_FLOAT, device=dev)
        lse2_all[world * B:].fill_(float("inf"))
        w_l = all_gather_rows(lse2_all[:world * B], lse2, group, async_op=True)
        ctx.works = (w_q, w_l)
        # internal buffers (not inputs or outputs), some still being filled by the async
        # all-gathers: kept on ctx rather than version-checked by save_for_backward
        ctx.bufs = (qb_all, lse2_all, db, dqu, ws) if want_grad else None
        ctx.meta = (B, M, H, dt, float(inv_tau), world, rank, float(1.0 / B) if grad_scale is None else float(grad_scale))
        ctx.group = group
        return loss

    @staticmethod
    def backward(ctx, g):
        qb_all, lse2_all, db, dqu, ws = ctx.bufs
        ctx.bufs = None
        B, M, H, dt, inv_tau, world, rank, grad_scale = ctx.meta
        for w in ctx.works:
            if w is not None:
                w.wait()
        ctx.works = ()
        g = g.to(_FLOAT).contiguous().reshape(1)
        g_kernel = g
        if _UNIFORM_SEED[0] == 0:
            lse2_all, g_kernel = _rank_seeds(lse2_all, g, B, world, ctx.group)
        dq = torch.empty(B, H, dtype=_FLOAT, device=db.device)
        dd = torch.empty(M, H, dtype=_FLOAT, device=db.device)
        call("tt_inbatch_bwd_ex", ptr(qb_all), ptr(lse2_all), world * B, rank * B, ptr(db), M, B, 0, H, dt, inv_tau,
             ptr(dqu), ptr(g_kernel), grad_scale, ptr(dq), ptr(dd), ptr(ws), ws.numel(), stream_of(db))
        if g_kernel is not g:  # this rank's own terms at its own seed (see _rank_seeds)
            dq.mul_(g / torch.where(g_kernel > 0, g_kernel, torch.ones_like(g_kernel)))
            lab = qb_all[rank * B:(rank + 1) * B].float()
            dd[:B].add_(lab * ((g_kernel - g) * (grad_scale * inv_tau)))
        return dq, dd, None, None, None, None


def in_batch_softmax_loss(q: torch.Tensor, d: torch.Tensor, temperature: float = 0.1, label_off: int = 0,
                          compute_dtype="fp32", grad_scale: float | None = None) -> torch.Tensor:
    return InBatchSoftmaxLoss.apply(q, d, 1.0 / float(temperature), label_off, compute_dtype, grad_scale)


# --------------------------------------------------------------------------------------------
# torch.optim.AdamW step (twotower/train.py:359, :139)
def adamw_step(param: torch.Tensor, grad: torch.Tensor, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor, *,
               lr: float, beta1: float, beta2: float, eps: float, weight_decay: float, step: int) -> None:
    require_gpu(param, grad, exp_avg, exp_avg_sq)
    for t, nm in ((param, "param"), (grad, "grad"), (exp_avg, "exp_avg"), (exp_avg_sq, "exp_avg_sq")):
        if not t.is_contiguous() or t.dtype != _FLOAT:
            raise ValueError(f"{nm} must be a contiguous float32 tensor")
    call("tt_adamw", ptr(param), ptr(grad), ptr(exp_avg), ptr(exp_avg_sq), param.numel(), lr, beta1, beta2, eps,
         weight_decay, step, stream_of(param))


def adam_prepare(slots: list[tuple[torch.Tensor, torch.Tensor]], *, lr: float, beta1: float, beta2: float, eps: float,
                 weight_decay: float, increment: int = 1, ahead: int = 0) -> None:
    """Device step += increment and the scalars of step + ahead for each (step, args) pair
    (tt_adam_prepare_ex; the defaults are tt_adam_prepare)."""
    if not slots:
        return
    stream = stream_of(slots[0][0])
    for i in range(0, len(slots), _lib.TT_ADAM_MAX_TENSORS):
        chunk = slots[i:i + _lib.TT_ADAM_MAX_TENSORS]
        arr = (_lib.AdamSlot * len(chunk))(*[_lib.AdamSlot(ptr(st), ptr(a)) for st, a in chunk])
        call("tt_adam_prepare_ex", arr, len(chunk), lr, beta1, beta2, eps, weight_decay, int(increment), int(ahead),
             stream)


def adamw_multi(items: list[tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]]) -> None:
    """(param, grad, exp_avg, exp_avg_sq, args) tensors updated in launches of up to 16."""
    if not items:
        return
    stream = stream_of(items[0][0])
    for i in range(0, len(items), _lib.TT_ADAM_MAX_TENSORS):
        chunk = items[i:i + _lib.TT_ADAM_MAX_TENSORS]
        arr = (_lib.AdamwTensor * len(chunk))(
            *[_lib.AdamwTensor(ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), ptr(a)) for p, g, m, v, a in chunk])
        call("tt_adamw_multi", arr, len(chunk), stream)


def pack_blocks(srcs, dst: torch.Tensor) -> None:
    """Contiguous device tensors copied into consecutive ranges of dst in one launch
    (tt_pack_blocks), on the current stream."""
    require_gpu(dst, *srcs)
    n = len(srcs)
    arr = (ctypes.c_void_p * max(n, 1))(*[ptr(t) for t in srcs])
    nb = (ctypes.c_int64 * max(n, 1))(*[t.numel() * t.element_size() for t in srcs])
    if sum(nb[:n]) > dst.numel() * dst.element_size():
        raise ValueError("pack_blocks: sources larger than the destination")
    call("tt_pack_blocks", arr, nb, n, ptr(dst), stream_of(dst))


def adamw_multi_ex(items, parts: list | None, next_slots: list, *, lr: float, beta1: float, beta2: float, eps: float,
                   weight_decay: float, ticket: torch.Tensor) -> None:
    """One tt_adamw_multi_ex launch (at most 16 tensors, 16 next slots): items as adamw_multi;
    parts[i] None or (part pointer, stride, slabs, owner) whose fixed-order sum becomes items[i]'s
    gradient; then the next step's scalars of next_slots (increment 1, ahead 1), formed by the
    launch's last workgroup: `ticket` is a zeroed device int32 tensor of at least
    TT_ADAM_TICKET_WORDS elements, left zeroed."""
    if len(items) > _lib.TT_ADAM_MAX_TENSORS or len(next_slots) > _lib.TT_ADAM_MAX_TENSORS:
        raise ValueError("adamw_multi_ex: at most 16 tensors and 16 slots per launch")
    if next_slots and (ticket.dtype != torch.int32 or ticket.numel() < _lib.TT_ADAM_TICKET_WORDS
                       or not ticket.is_contiguous()):
        raise ValueError(f"adamw_multi_ex: ticket must be {_lib.TT_ADAM_TICKET_WORDS} contiguous int32 words")
    if not items and not next_slots:
        return
    stream = stream_of(items[0][0] if items else next_slots[0][0])
    n = max(len(items), 1)
    arr = (_lib.AdamwTensor * n)(
        *[_lib.AdamwTensor(ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), ptr(a)) for p, g, m, v, a in items])
    gp = (_lib.AdamwGradParts * n)()
    for i, pt in enumerate(parts or []):
        if pt is not None:
            gp[i] = _lib.AdamwGradParts(pt[0], pt[1], pt[2])
    sl = (_lib.AdamSlot * max(len(next_slots), 1))(*[_lib.AdamSlot(ptr(st), ptr(a)) for st, a in next_slots])
    call("tt_adamw_multi_ex", arr, gp, len(items), sl, len(next_slots), lr, beta1, beta2, eps, weight_decay,
         ptr(ticket), stream)


def bag_mean_backward_adamw_planned(d_pooled, denom, plan: BagPlan, table, exp_avg, exp_avg_sq,
                                    adam_args: torch.Tensor) -> None:
    """Fused scatter + AdamW from a BagPlan, per-step scalars read from device memory."""
    d_pooled = _contig_f32(d_pooled, "d_pooled")
    if table.shape[0] != plan.V or table.shape[1] != plan.E:
        raise ValueError("plan was built for a different table shape")
    plan.wait()
    call("tt_bag_mean_bwd_adamw_planned", ptr(d_pooled), ptr(denom), plan.nseq, plan.L, plan.V, plan.E, ptr(plan.buf),
         plan.buf.numel(), ptr(table), ptr(exp_avg), ptr(exp_avg_sq), ptr(adam_args), stream_of(table))


def bag_mean_backward_adamw_planned_rows(d_pooled, denom, plan: BagPlan, row_begin: int, row_end: int, table_rows,
                                         exp_avg_rows, exp_avg_sq_rows, adam_args: torch.Tensor) -> None:
    """Rows [row_begin, row_end) of the fused scatter + AdamW (after bag_mean_backward_planned_prepare on the
    same stream): table_rows, exp_avg_rows, exp_avg_sq_rows are those rows ((row_end - row_begin, E))."""
    d_pooled = _contig_f32(d_pooled, "d_pooled")
    n = row_end - row_begin
    for t, nm in ((table_rows, "table_rows"), (exp_avg_rows, "exp_avg_rows"), (exp_avg_sq_rows, "exp_avg_sq_rows")):
        if tuple(t.shape) != (n, plan.E) or not t.is_contiguous() or t.dtype != _FLOAT:
            raise ValueError(f"{nm} must be a contiguous float32 ({n}, {plan.E}) tensor")
    call("tt_bag_mean_bwd_adamw_planned_rows", ptr(d_pooled), ptr(denom), plan.nseq, plan.L, plan.V, plan.E,
         ptr(plan.buf), plan.buf.numel(), int(row_begin), int(row_end), ptr(table_rows), ptr(exp_avg_rows),
         ptr(exp_avg_sq_rows), ptr(adam_args), stream_of(table_rows))


def bag_mean_backward_adamw(d_pooled, denom, ids, table, exp_avg, exp_avg_sq, padding_idx, *, lr, beta1, beta2,
                            eps, weight_decay, step) -> None:
    """Sorted scatter of the pooled gradient fused with the table's AdamW step."""
    d_pooled = _contig_f32(d_pooled, "d_pooled")
    N, E = d_pooled.shape
    V = table.shape[0]
    L = ids.shape[1]
    dev = table.device
    nbytes = _lib.lib().tt_bag_mean_bwd_ws_size(N, L, V, E)
    ws = WORKSPACE.get("bag_bwd", nbytes, dev)
    pad = -1 if padding_idx is None else int(padding_idx)
    call("tt_bag_mean_bwd_adamw", ptr(d_pooled), ptr(denom), ptr(ids), _lib.ids_dtype_code(ids), N, L, L, V, E,
         pad, ptr(table), ptr(exp_avg), ptr(exp_avg_sq), lr, beta1, beta2, eps, weight_decay, step, ptr(ws),
         ws.numel(), stream_of(table))


# --------------------------------------------------------------------------------------------
# search: cosine scores + top-k   (inference/search/two_tower.py:92-103, evaluate.py:176-183)
def cosine_scores(q: torch.Tensor, docs: torch.Tensor) -> torch.Tensor:
    """(nq, nd) F.cosine_similarity(q_i, d_j) (eps 1e-8) on the HBM-streaming HIP kernel."""
    require_gpu(q, docs)
    q, docs = _contig_f32(q, "q"), _contig_f32(docs, "docs")
    if q.dim() == 1:
        q = q.unsqueeze(0)
    nq, H = q.shape
    if docs.shape[1] != H:
        raise ValueError(f"query width {H} != document width {docs.shape[1]}")
    out = torch.empty(nq, docs.shape[0], dtype=_FLOAT, device=q.device)
    call("tt_cosine_scores", ptr(q), nq, ptr(docs), docs.shape[0], H, ptr(out), stream_of(q))
    return out


def topk_rows(scores: torch.Tensor, k: int) -> tuple[torch.Tensor, torch.Tensor]:
    """torch.topk(scores, k, dim=1) (descending; ties to the lower index) on the HIP radix select."""
    require_gpu(scores)
    scores = _contig_f32(scores, "scores")
    if scores.dim() == 1:
        scores = scores.unsqueeze(0)
    n, m = scores.shape
    vals = torch.empty(n, k, dtype=_FLOAT, device=scores.device)
    idx = torch.empty(n, k, dtype=torch.int64, device=scores.device)
    nbytes = _lib.lib().tt_topk_rows_ws_size(n, m, int(k))
    ws = WORKSPACE.get("topk", nbytes, scores.device) if nbytes else None
    call("tt_topk_rows_ex", ptr(scores), n, m, int(k), ptr(ws) if ws is not None else None, nbytes, ptr(vals),
         ptr(idx), stream_of(scores))
    return vals, idx


def cosine_topk(q: torch.Tensor, docs: torch.Tensor, k: int) -> tuple[torch.Tensor, torch.Tensor]:
    return topk_rows(cosine_scores(q, docs), k)
