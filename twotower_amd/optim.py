"""AdamW on the HIP kernels: the same update as torch.optim.AdamW (twotower/train.py:359,
stepped at :139; defaults lr 1e-3, betas (0.9, 0.999), eps 1e-8, weight_decay 1e-2), with the
same per-parameter state keys ('step', 'exp_avg', 'exp_avg_sq') so optimizer state_dicts
interchange.

``fused_tables=True`` lets the embedding tables skip their dense V x E gradient: the bag
backward leaves its factored gradient (ids, d_pooled, denom, sort plan) on the table and
``step`` runs the sorted scatter fused with the AdamW update.  The result equals the dense path
exactly in math (every row is decayed and its moments updated, rows without tokens with g = 0),
it just never writes or re-reads the dense gradient.

``capturable=True`` follows torch's convention of the same name: each ``state['step']`` lives on
the parameter's device and is advanced there (tt_adam_prepare), the per-step scalars are read
from device memory, and the small parameters are updated by one multi-tensor launch, so a whole
training step can be captured in a HIP graph and replayed (train_step.TrainStep(graph=True)).
"""
from __future__ import annotations

import math
import os
import weakref

import torch
import torch.nn.functional as F

from . import _lib, distributed, ops


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 1e-2,
                 fused_tables: bool = False, tables=(), capturable: bool = False, group=None,
                 table_sync: str = "auto"):
        if lr < 0.0 or eps < 0.0 or weight_decay < 0.0:
            raise ValueError("invalid AdamW hyper-parameter")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay,
                                      capturable=bool(capturable)))
        self._tables: list[torch.Tensor] = []
        self._side_grads = _lib.SideGrads()
        self._grad_sync = None  # distributed.GradSync set by train_step.TrainStep around its step(): launched inside
        self._sync_todo = False
        self._backward_done = None
        self._args: dict[int, torch.Tensor] = {}  # id(param) -> device per-step scalars (capturable)
        self._shards: dict[int, distributed.ShardedRows] = {}  # data parallel: row-sharded tables
        self._columns: dict[int, distributed.ColumnTable] = {}  # data parallel: column-sharded tables
        # moment tensors already in the sharded layout (by identity; weak, so loaded state replaces them)
        self._sharded_moments: dict[int, weakref.ref] = {}
        # capturable: id(step tensor) -> (hyper-parameters, that tensor) of the args formed one step
        # ahead by the previous step's tail launch; see _step_device
        self._ahead: dict[int, tuple] = {}
        self._tickets: dict[torch.device, torch.Tensor] = {}  # tt_adamw_multi_ex's last-workgroup ticket
        if fused_tables:
            ids = {id(p) for g in self.param_groups for p in g["params"]}
            for t in tables:
                inner = getattr(t, "embedding", None)
                w = inner.weight if inner is not None else t
                pad = getattr(inner, "padding_idx", 0) if inner is not None else 0
                if id(w) not in ids:
                    raise ValueError("fused table is not among the optimizer's parameters")
                mode = distributed.table_sync_mode(table_sync, group, E=w.shape[1])
                # (None is the "no exchange" sentinel there: name the default group explicitly)
                gg = ((group if group is not None else torch.distributed.group.WORLD) if mode in ("gather", "owner")
                      else None)
                w._tt_deferred = ops.DeferredTableGrad(pad, gather_group=gg)
                self._tables.append(w)
                if mode in ("shard", "owner"):  # owner: shard's row partition, gather's inputs
                    self._shards[id(w)] = distributed.ShardedRows(w, group)
                elif mode == "column":  # each rank owns E / world columns of every row (its slab)
                    col = distributed.ColumnTable(w, group, module=inner if inner is not None else None)
                    self._columns[id(w)] = w._tt_column = col
            # the dense parameters' gradients may then be computed on a side stream beside the
            # fused table update (ops.TowerHead); step() joins them after launching that update
            tabs = {id(w) for w in self._tables}
            for g in self.param_groups:
                for p in g["params"]:
                    if id(p) not in tabs:
                        p._tt_side_grads = self._side_grads

    def release_tables(self) -> None:
        """Return the tables to ordinary dense gradients (and every gradient to the current stream);
        a column-sharded table is materialized first and a sharded table's moments are gathered to
        the full table (both collective), so the next dense step updates V x E moments."""
        for w in self._tables:
            if hasattr(w, "_tt_deferred"):
                del w._tt_deferred
            col = self._columns.pop(id(w), None)
            sh = self._shards.pop(id(w), None)
            st = self.state.get(w)
            if col is not None:
                col.materialize()
                del w._tt_column
            if st and (col is not None or sh is not None):
                for k in ("exp_avg", "exp_avg_sq"):
                    m = st[k]
                    self._sharded_moments.pop(id(m), None)
                    full = col.gather_cols(m) if col is not None else sh.gather_full(m)[:w.shape[0]]
                    st[k] = full.contiguous().clone()
        self._tables = []
        for g in self.param_groups:
            for p in g["params"]:
                if getattr(p, "_tt_side_grads", None) is self._side_grads:
                    del p._tt_side_grads
        self._side_grads.join()

    def _state(self, p: torch.Tensor, capturable: bool) -> dict:
        st = self.state[p]
        if not st:
            st["step"] = torch.tensor(0.0, dtype=torch.float32, device=p.device if capturable else "cpu")
            sh = self._shards.get(id(p))
            col = self._columns.get(id(p))
            like = (p if sh is None else p.new_empty(sh.Vs, sh.E)) if col is None else col.slab  # own rows / columns
            st["exp_avg"] = torch.zeros_like(like, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(like, memory_format=torch.preserve_format)
            if sh is not None or col is not None:
                self._mark_sharded(st["exp_avg"])
        else:
            if capturable and st["step"].device != p.device:
                st["step"] = st["step"].to(device=p.device, dtype=torch.float32)
            col = self._columns.get(id(p))
            if col is not None and not self._is_sharded(st["exp_avg"]):  # full-table moments loaded: own columns
                for k in ("exp_avg", "exp_avg_sq"):
                    if tuple(st[k].shape) != (col.V, col.E):
                        raise ValueError(f"column table state: {k} has shape {tuple(st[k].shape)}, expected "
                                         f"{(col.V, col.E)}")
                    st[k] = col.own_cols(st[k].to(col.slab.device))
                self._mark_sharded(st["exp_avg"])
            sh = self._shards.get(id(p))
            # full-table moments loaded (load_state_dict): keep this rank's rows.  Told apart from
            # the moments this optimizer sharded itself by identity, not by shape: at one rank the
            # shard has the table's own row count (a shape test re-sharded them on every step,
            # which a captured step then replayed from stale copies)
            if sh is not None and not self._is_sharded(st["exp_avg"]):
                for k in ("exp_avg", "exp_avg_sq"):
                    if st[k].shape[0] != sh.V:
                        raise ValueError(f"sharded table state: {k} has {st[k].shape[0]} rows, expected {sh.V}")
                    full = torch.zeros(sh.Vp, sh.E, dtype=st[k].dtype, device=st[k].device)
                    full[:sh.V] = st[k]
                    st[k] = sh.rows(full).clone()
                self._mark_sharded(st["exp_avg"])
        return st

    def _mark_sharded(self, t: torch.Tensor) -> None:
        self._sharded_moments[id(t)] = weakref.ref(t)

    def _is_sharded(self, t: torch.Tensor) -> bool:
        r = self._sharded_moments.get(id(t))
        return r is not None and r() is t

    def state_dict(self):
        """torch's layout; a row-sharded table (data parallel "shard" sync) reports its full-size
        moments (all-gathered over the ranks), so the state loads into torch.optim.AdamW and
        into a differently sharded run."""
        sd = super().state_dict()
        if not self._shards and not self._columns:
            return sd
        index = {id(p): i for i, p in enumerate(p for g in self.param_groups for p in g["params"])}
        for p in (p for g in self.param_groups for p in g["params"]):
            sh = self._shards.get(id(p))
            col = self._columns.get(id(p))
            st = sd["state"].get(index[id(p)])
            if (sh is None and col is None) or st is None:
                continue
            st = sd["state"][index[id(p)]] = dict(st)  # the packed dict aliases the live state
            for k in ("exp_avg", "exp_avg_sq"):
                st[k] = sh.gather_full(st[k])[:sh.V].clone() if sh is not None else col.gather_cols(st[k])
        return sd

    def load_state_dict(self, state_dict) -> None:
        """torch semantics, except that `capturable` stays what this optimizer was built with (it
        selects the execution path, not the math); step counters move on first use."""
        modes = [g["capturable"] for g in self.param_groups]
        self._ahead.clear()  # scalars formed ahead belong to the replaced counters
        super().load_state_dict(state_dict)
        for g, c in zip(self.param_groups, modes):
            g["capturable"] = c

    def _adam_args(self, p: torch.Tensor) -> torch.Tensor:
        a = self._args.get(id(p))
        if a is None:
            a = self._args[id(p)] = torch.zeros(_lib.TT_ADAM_ARGS_BYTES // 4, dtype=torch.float32, device=p.device)
        return a

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        # The tower-gradient all-reduce (data parallel, set by TrainStep for its step) runs once
        # per step whatever the number of param groups; the communication stream waits for this
        # point of the current stream (the end of backward), not for the table update queued next.
        self._sync_todo = self._grad_sync is not None
        self._backward_done = None
        if self._sync_todo and torch.cuda.is_available() and any(
                p.is_cuda for g in self.param_groups for p in g["params"]):
            self._backward_done = torch.cuda.Event()
            self._backward_done.record()
        try:
            for group in self.param_groups:
                if group["capturable"]:
                    self._step_device(group)
                else:
                    self._step_host(group)
        finally:
            self._sync_todo = False
            self._backward_done = None
        return loss

    def _launch_grad_sync(self) -> None:
        """Launch the all-reduce of the dense gradients, once per step (see step)."""
        if getattr(self, "_sync_todo", False):
            self._sync_todo = False
            self._grad_sync.launch(self._side_grads, after=self._backward_done)

    def _step_host(self, group: dict) -> None:
        """torch's default (non-capturable) form: step counters on the host."""
        lr, (b1, b2), eps, wd = group["lr"], group["betas"], group["eps"], group["weight_decay"]
        self._launch_grad_sync()
        self._side_grads.join()
        for p in group["params"]:
            deferred = getattr(p, "_tt_deferred", None)
            if deferred is not None and deferred.parts:
                st = self._state(p, False)
                st["step"] += 1
                col = self._columns.get(id(p))
                if col is not None:  # "column": this rank's slab from every rank's factored gradient
                    args = _host_adam_args(lr, b1, b2, eps, wd, int(st["step"]), p.device)
                    ops.bag_col_update(col, list(deferred.parts), st["exp_avg"], st["exp_avg_sq"], args)
                    deferred.parts.clear()
                    continue
                ids, dp, den, plan = _merge_parts(deferred.parts, p, deferred.padding_idx)
                deferred.parts.clear()
                if deferred.gather_group is not None:
                    ids, dp, den, plan = _gather_parts((ids, dp, den, plan), deferred.gather_group)
                sh = self._shards.get(id(p))
                if sh is not None:
                    args = _host_adam_args(lr, b1, b2, eps, wd, int(st["step"]), p.device)
                    upd = self._owner_update if deferred.gather_group is not None else self._shard_update
                    upd(sh, (ids, dp, den, plan), st, args)
                    torch.cuda.current_stream(p.device).wait_stream(sh.comm_stream())
                    continue
                args = _host_adam_args(lr, b1, b2, eps, wd, int(st["step"]), p.device)
                ops.bag_mean_backward_adamw_planned(dp, den, plan, p.data, st["exp_avg"], st["exp_avg_sq"], args)
                continue
            if p.grad is None:
                continue
            if p.grad.is_sparse:
                raise RuntimeError("AdamW does not support sparse gradients")
            st = self._state(p, False)
            _check_dense_moments(p, st)
            st["step"] += 1
            ops.adamw_step(p.data, p.grad.contiguous(), st["exp_avg"], st["exp_avg_sq"], lr=lr, beta1=b1,
                           beta2=b2, eps=eps, weight_decay=wd, step=int(st["step"]))

    def _step_device(self, group: dict) -> None:
        """Capturable form: one tt_adam_prepare launch, one multi-tensor launch per 16 dense
        parameters, one fused scatter + AdamW launch per table."""
        slots, dense, fused, shards, dense_ids, columns = [], [], [], [], [], []
        for p in group["params"]:
            deferred = getattr(p, "_tt_deferred", None)
            if deferred is not None and deferred.parts:
                st = self._state(p, True)
                a = self._adam_args(p)
                slots.append((st["step"], a))
                col = self._columns.get(id(p))
                if col is not None:  # "column": every rank's factored gradient at this rank's columns
                    columns.append((col, list(deferred.parts), st, a))
                    deferred.parts.clear()
                    continue
                parts = _merge_parts(deferred.parts, p, deferred.padding_idx)
                deferred.parts.clear()
                sh = self._shards.get(id(p))
                if sh is not None and deferred.gather_group is not None:  # "owner": every rank's factored
                    # gradient, this rank's rows updated, the rows all-gathered in chunks
                    shards.append((sh, _gather_parts(parts, deferred.gather_group), st, a, self._owner_update))
                elif sh is not None:  # data parallel: chunked reduce-scatter, AdamW on own rows, all-gather
                    shards.append((sh, parts, st, a, self._shard_update))
                else:
                    if deferred.gather_group is not None:  # data parallel: every rank's factored grad
                        parts = _gather_parts(parts, deferred.gather_group)
                    fused.append((p, st, parts))
                continue
            if p.grad is None:
                continue
            if p.grad.is_sparse:
                raise RuntimeError("AdamW does not support sparse gradients")
            for t, nm in ((p, "param"), (p.grad, "grad")):
                if not t.is_cuda or t.dtype != torch.float32:
                    raise ValueError(f"capturable AdamW needs float32 GPU tensors ({nm} is {t.dtype} on {t.device})")
            st = self._state(p, True)
            _check_dense_moments(p, st)
            a = self._adam_args(p)
            slots.append((st["step"], a))
            dense.append((p.data, p.grad.contiguous(), st["exp_avg"], st["exp_avg_sq"], a))
            dense_ids.append(id(p))
        if not slots:  # nothing to update in this group (frozen, unused, or no backward): torch does nothing
            self._launch_grad_sync()
            return
        lr, (b1, b2), eps, wd = group["lr"], group["betas"], group["eps"], group["weight_decay"]
        hyper = (lr, b1, b2, eps, wd)
        # Scalars one step ahead (TT_ADAM_AHEAD=0: torch's order, a prepare in front of the
        # updates): the previous step's tail formed this step's scalars while advancing its counters
        # (tt_adam_prepare_ex increment 1, ahead 1), so the fused table update follows the
        # backward directly instead of waiting on a prepare launched after it.  Counters nobody
        # prepared, or prepared with other hyper-parameters, get theirs here (increment 0, ahead 1).
        ahead = os.environ.get("TT_ADAM_AHEAD", "1") != "0"
        if ahead:
            def warm(st):
                h, t = self._ahead.get(id(st), (None, None))
                return t is st and h == hyper

            cold = [sl for sl in slots if not warm(sl[0])]
            ops.adam_prepare(cold, lr=lr, beta1=b1, beta2=b2, eps=eps, weight_decay=wd, increment=0, ahead=1)
        else:
            for st, _ in slots:
                self._ahead.pop(id(st), None)
            ops.adam_prepare(slots, lr=lr, beta1=b1, beta2=b2, eps=eps, weight_decay=wd)
        # the fused table updates first: they read no dense gradient, so side-stream gradients
        # (ops.TowerHead's weight gradients) are still being computed beside them
        for p, st, (ids, dp, den, plan) in fused:
            ops.bag_mean_backward_adamw_planned(dp, den, plan, p.data, st["exp_avg"], st["exp_avg_sq"],
                                                self._adam_args(p))
        for col, parts, st, a in columns:  # column-sharded tables: this rank's slab, no exchange left
            ops.bag_col_update(col, parts, st["exp_avg"], st["exp_avg_sq"], a)
        # data parallel, row-sharded tables: the chunk-pipelined exchange (its collectives are
        # issued before the tower all-reduce, so they lead on the communicator)
        for sh, parts, st, a, update in shards:
            update(sh, parts, st, a)

        def join_shards():  # the chunk updates read this step's scalars on their own stream: the
            for sh, _, _, _, _ in shards:  # next step's scalars (and the next forward) wait for them
                torch.cuda.current_stream(sh.weight.device).wait_stream(sh.comm_stream())
        # data parallel: the tower-gradient all-reduce, issued after the table's collectives and
        # the table update, overlaps that update on a communication stream; the join waits for it
        self._launch_grad_sync()
        # The step's tail (TT_FUSED_TAIL=0: the slab sums as their own launch): the dense updates
        # form the head weight gradients from their side-stream slab partials themselves (the sums
        # of tt_head_wgrad2_reduce, bit for bit, also written to .grad; tt_adamw_multi_ex).  The
        # next step's scalars stay a launch of their own: formed by the same launch's last
        # workgroup (two-level ticket) the step measured the same, 0.8446-0.8486 against
        # 0.8407-0.8484 ms (profiles/r06s_prepare_in_tail_ab.txt; round 2's single counter cost more).
        fuse = (os.environ.get("TT_FUSED_TAIL", "1") != "0" and len(dense) <= _lib.TT_ADAM_MAX_TENSORS
                and len(slots) <= _lib.TT_ADAM_MAX_TENSORS and (dense or ahead))
        parts = self._side_grads.join(claim={i for i in dense_ids if i is not None} if fuse else None)
        if fuse:
            dev = (dense[0][0] if dense else slots[0][0]).device
            ticket = self._tickets.get(dev)
            if ticket is None:
                ticket = self._tickets[dev] = torch.zeros(_lib.TT_ADAM_TICKET_WORDS, dtype=torch.int32, device=dev)
            ops.adamw_multi_ex(dense, [parts.get(i) if i is not None else None for i in dense_ids], [], lr=lr,
                               beta1=b1, beta2=b2, eps=eps, weight_decay=wd, ticket=ticket)
            join_shards()
            if ahead:
                ops.adam_prepare(slots, lr=lr, beta1=b1, beta2=b2, eps=eps, weight_decay=wd, increment=1, ahead=1)
        else:
            ops.adamw_multi(dense)
            join_shards()
            if ahead:  # counters advanced, next step's scalars formed, behind every update that read them
                ops.adam_prepare(slots, lr=lr, beta1=b1, beta2=b2, eps=eps, weight_decay=wd, increment=1, ahead=1)
        if ahead:
            for st, _ in slots:
                self._ahead[id(st)] = (hyper, st)  # the tensor itself: an id alone could be reused

    @staticmethod
    def _shard_update(sh, parts, st, args) -> None:
        """Row-sharded table update under data parallelism (the loss is pre-scaled by 1/world, so
        the reduce-scattered sums are global-batch mean gradients), pipelined over the row chunks
        of ShardedRows: the current stream forms chunk c's dense gradient rows
        (tt_bag_mean_bwd_planned_rows) and hands them to the communication stream, which
        reduce-scatters them, runs AdamW on this rank's slab (moments: its chunk of the sharded
        state) and all-gathers the updated slab into every rank's table, while the current stream
        goes on with chunk c + 1.  The caller joins sh.comm_stream() before anything reads the
        table or the step scalars `args` again."""
        _, dp, den, plan = parts
        dev = dp.device
        main = torch.cuda.current_stream(dev)
        comm = sh.comm_stream()
        gbuf, gsh = sh.step_buffers()
        stor = sh.storage()
        ops.bag_mean_backward_planned_prepare(dp, den, plan)
        for c in range(sh.NC):
            lo, hi = sh.chunk(c)
            top = min(hi, sh.V)
            if lo < top:
                ops.bag_mean_backward_planned_rows(dp, den, plan, lo, top, gbuf[lo:top])
            ready = torch.cuda.Event()
            ready.record(main)
            comm.wait_event(ready)
            with torch.cuda.stream(comm):
                g = sh.shard_chunk(gsh, c)
                distributed.reduce_scatter_rows(g, gbuf[lo:hi], sh.group)
                ops.adamw_multi([(sh.own(stor, c), g, sh.shard_chunk(st["exp_avg"], c),
                                  sh.shard_chunk(st["exp_avg_sq"], c), args)])
                distributed.all_gather_rows(stor[lo:hi], sh.own(stor, c), sh.group)


    @staticmethod
    def _owner_update(sh, parts, st, args) -> None:
        """Row-owner table update ("owner" exchange): `parts` is every rank's factored gradient
        (all-gathered ids in the plan, d_pooled / denom), so this rank forms the global gradient of
        exactly the rows it owns and applies AdamW to them with its moment shard
        (tt_bag_mean_bwd_adamw_planned_rows, the fused update's sums and order for those rows), chunk
        by chunk; the communication stream all-gathers chunk c's owned slabs into every rank's table
        while the current stream updates chunk c + 1.  No dense gradient and no reduce-scatter; the
        caller joins sh.comm_stream() before the table or `args` are read again."""
        _, dp, den, plan = parts
        main = torch.cuda.current_stream(dp.device)
        comm = sh.comm_stream()
        stor = sh.storage()
        ops.bag_mean_backward_planned_prepare(dp, den, plan)
        for c in range(sh.NC):
            lo = c * sh.Cr + sh.rank * sh.R
            top = min(lo + sh.R, sh.V)
            if lo < top:
                n = top - lo
                ops.bag_mean_backward_adamw_planned_rows(dp, den, plan, lo, top, stor[lo:top],
                                                         sh.shard_chunk(st["exp_avg"], c)[:n],
                                                         sh.shard_chunk(st["exp_avg_sq"], c)[:n], args)
            ready = torch.cuda.Event()
            ready.record(main)
            comm.wait_event(ready)
            with torch.cuda.stream(comm):
                clo, chi = sh.chunk(c)
                distributed.all_gather_rows(stor[clo:chi], sh.own(stor, c), sh.group)


class BackwardTableUpdate:
    """The fused table update for a loop that keeps ``torch.optim.AdamW`` (the reference's
    ``train.py:359``, stepped at ``:139``): at the end of every ``loss.backward()`` the table's
    factored gradient goes through the sorted scatter fused with AdamW
    (tt_bag_mean_bwd_adamw_planned) with the hyper-parameters of the table's param group in that
    optimizer, and the table never gets a ``.grad``, so ``optimizer.step()`` skips it (torch's
    AdamW steps only parameters with a gradient) and updates the tower parameters as before.

    The moments and step counter live in ``optimizer.state[table]`` under torch's own keys
    ('step' a CPU float32 tensor, 'exp_avg', 'exp_avg_sq'), so ``optimizer.state_dict()``,
    ``save_checkpoint`` / ``load_checkpoint`` (utils.py:231-330) and a later switch back to the
    plain path all see the same state.  The arithmetic is the fused update's, checked against
    torch.optim.AdamW elementwise (tests).  What differs from torch's order of events: the table is
    updated inside backward (once per backward pass), so a loop that accumulates several
    backwards per optimizer step, or skips a step, must not use it; train.py does neither."""

    def __init__(self, optimizer: torch.optim.Optimizer, weight: torch.Tensor, padding_idx: int | None = 0):
        if not isinstance(optimizer, torch.optim.AdamW) or isinstance(optimizer, AdamW):
            raise TypeError("table_update 'backward' drives a torch.optim.AdamW the loop keeps "
                            f"(twotower_amd.optim.AdamW(fused_tables=True) fuses it itself); got {type(optimizer).__name__}")
        self.optimizer = optimizer
        self.weight = weight
        self._check(self.group)
        if getattr(weight, "_tt_deferred", None) is not None:
            raise ValueError("the table's gradient is already owned by a fused optimizer")
        weight._tt_deferred = ops.DeferredTableGrad(padding_idx, on_backward=self)

    @property
    def group(self) -> dict:
        """The table's param group, looked up each time (load_state_dict replaces the group dicts)."""
        return _group_of(self.optimizer, self.weight)

    @staticmethod
    def _check(group: dict) -> None:
        for k in ("amsgrad", "maximize", "differentiable"):
            if group.get(k, False):
                raise ValueError(f"table_update 'backward' implements AdamW without {k}")
        if group.get("capturable", False) or group.get("fused", False):
            raise ValueError("table_update 'backward' keeps torch's host step counter (capturable=False, fused=False)")

    def release(self) -> None:
        """Back to the dense table gradient stepped by the optimizer (the state stays valid)."""
        if getattr(self.weight, "_tt_deferred", None) is not None and self.weight._tt_deferred.on_backward is self:
            del self.weight._tt_deferred

    @torch.no_grad()
    def __call__(self) -> None:
        w = self.weight
        deferred = w._tt_deferred
        if not deferred.parts:
            return
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("table_update 'backward' runs eagerly (host step counter); use TrainStep with "
                               "twotower_amd.optim.AdamW(capturable=True) for a captured step")
        g = self.group
        self._check(g)  # (a param group's options can be changed between steps)
        ids, dp, den, plan = _merge_parts(deferred.parts, w, deferred.padding_idx)
        deferred.parts.clear()
        st = _torch_adamw_state(self.optimizer, w)  # torch.optim.AdamW's _init_group layout
        st["step"] += 1
        b1, b2 = g["betas"]
        lr = float(g["lr"])
        args = _host_adam_args(lr, b1, b2, g["eps"], g["weight_decay"], int(st["step"]), w.device)
        ops.bag_mean_backward_adamw_planned(dp, den, plan, w.data, st["exp_avg"], st["exp_avg_sq"], args)


def _group_of(optimizer: torch.optim.Optimizer, p: torch.Tensor) -> dict:
    g = next((g for g in optimizer.param_groups if any(q is p for q in g["params"])), None)
    if g is None:
        raise ValueError("the parameter is not among the optimizer's parameters")
    return g


def _torch_adamw_state(optimizer: torch.optim.Optimizer, p: torch.Tensor) -> dict:
    """optimizer.state[p] in torch.optim.AdamW's non-capturable layout (step a CPU float32 tensor)."""
    st = optimizer.state[p]
    if not st:
        st["step"] = torch.tensor(0.0, dtype=torch.float32)
        st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
    return st


class BackwardDenseUpdate:
    """The companion of BackwardTableUpdate for the dense (tower) parameters of the same
    ``torch.optim.AdamW`` (config ``hip: {dense_update: backward}``): once every parameter's
    gradient of a ``loss.backward()`` has been accumulated, one multi-tensor AdamW launch
    (tt_adamw_multi, 16 tensors per launch) steps them all with their groups' hyper-parameters and
    the moments in ``optimizer.state[p]`` (torch's keys and layout), then drops their ``.grad``,
    so ``optimizer.step()`` finds nothing left to do.  torch's foreach AdamW is ~10 launches over
    the same bytes (108 us per C3 step on the GPU, profiles/r05i_plain_profile.txt, against a few
    us here).  Same caveat as the table: one backward per optimizer step, and nothing may read the
    parameters' ``.grad`` between ``backward()`` and ``step()`` (train.py:137-139 does neither)."""

    def __init__(self, optimizer: torch.optim.Optimizer, params):
        if not isinstance(optimizer, torch.optim.AdamW) or isinstance(optimizer, AdamW):
            raise TypeError(f"dense_update 'backward' drives a torch.optim.AdamW; got {type(optimizer).__name__}")
        self.optimizer = optimizer
        self.params = []
        for p in params:
            if not p.requires_grad or getattr(p, "_tt_deferred", None) is not None:
                continue
            BackwardTableUpdate._check(_group_of(optimizer, p))
            self.params.append(p)
        self._ids = {id(p) for p in self.params}
        self._queued = False
        self._handles = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]

    def _on_grad(self, _p) -> None:
        if not self._queued:
            self._queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._run)

    @torch.no_grad()
    def _run(self) -> None:
        self._queued = False
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("dense_update 'backward' runs eagerly (host step counter)")
        items, done, args_for = [], [], {}
        for g in self.optimizer.param_groups:
            BackwardTableUpdate._check(g)
            b1, b2 = g["betas"]
            for p in g["params"]:
                if id(p) not in self._ids or p.grad is None:
                    continue
                if p.grad.is_sparse or p.dtype != torch.float32:
                    raise RuntimeError("dense_update 'backward' steps dense float32 parameters")
                st = _torch_adamw_state(self.optimizer, p)
                st["step"] += 1
                key = (id(g), int(st["step"]))
                if key not in args_for:
                    args_for[key] = _host_adam_args(float(g["lr"]), b1, b2, g["eps"], g["weight_decay"], key[1],
                                                    p.device)
                items.append((p.data, p.grad.contiguous(), st["exp_avg"], st["exp_avg_sq"], args_for[key]))
                done.append(p)
        ops.adamw_multi(items)
        for p in done:
            p.grad = None

    def release(self) -> None:
        for h in self._handles:
            h.remove()
        self._handles = []


def fuse_dense_update(optimizer: torch.optim.Optimizer, model: torch.nn.Module) -> BackwardDenseUpdate:
    """Attach a BackwardDenseUpdate to every dense parameter of ``model`` the loop's own
    torch.optim.AdamW steps (the tables are fuse_table_update's).  The opt-in behind
    ``hip: {dense_update: backward}`` (twotower_amd.install)."""
    if getattr(optimizer, "_tt_dense_update", None) is not None:
        raise ValueError("the optimizer's dense parameters already have a backward update")
    upd = optimizer._tt_dense_update = BackwardDenseUpdate(optimizer, [p for p in model.parameters()])
    return upd


def fuse_table_update(optimizer: torch.optim.Optimizer, model_or_tables) -> list[BackwardTableUpdate]:
    """Attach a BackwardTableUpdate to every lookup table of ``model_or_tables`` (a model, an
    embedding, or a list of them; shared tables once) for the loop's own torch.optim.AdamW.
    The opt-in behind the reference config's ``hip: {table_update: backward}`` (twotower_amd.install)."""
    items = model_or_tables if isinstance(model_or_tables, (list, tuple)) else [model_or_tables]
    seen, out = set(), []
    for item in items:
        mods = item.modules() if isinstance(item, torch.nn.Module) else [item]
        for m in mods:
            inner = getattr(m, "embedding", None)
            if not isinstance(inner, torch.nn.Embedding) or id(inner.weight) in seen:
                continue
            seen.add(id(inner.weight))
            out.append(BackwardTableUpdate(optimizer, inner.weight, inner.padding_idx))
    if not out:
        raise ValueError("no lookup table (an nn.Embedding at .embedding) found")
    return out


def _gather_parts(parts, group):
    """Replicated table update under data parallelism: all-gather d_pooled and denom (rank-major,
    matching the plan's all-gathered ids); with the loss pre-scaled by 1/world the sum over all
    ranks' entries is the global-batch mean gradient, applied identically on every rank."""
    ids, dp, den, plan = parts
    world = torch.distributed.get_world_size(group)
    dp_all = dp.new_empty((world * dp.shape[0],) + tuple(dp.shape[1:]))
    distributed.all_gather_rows(dp_all, dp.contiguous(), group)
    den_all = None  # None: d_pooled arrived divided by its denominators (ops.bag_head_prescale)
    if den is not None:
        den_all = den.new_empty((world * den.shape[0],))
        distributed.all_gather_rows(den_all, den.contiguous(), group)
    if plan is None or plan.nseq != dp_all.shape[0]:
        raise RuntimeError("replicated table sync needs the all-ranks plan built in the forward")
    return plan.ids, dp_all, den_all, plan


class _ArgsRing:
    """Host-to-device staging of the per-step AdamW scalars without a host sync: a pageable
    ``torch.tensor(...).to(device)`` is a blocking copy ordered behind everything queued on the
    stream, i.e. a full drain in the middle of the step (the unchanged train.py loop issues its
    next kernels only after it).  The scalars go into one of a ring of pinned buffers and are
    copied on the current stream (non_blocking); a buffer is rewritten only once its last copy
    has executed (its event, long complete by then in practice)."""

    def __init__(self, n: int = 16):
        self.n, self.k = n, 0
        self.host = self.host_np = None
        self.events: list = [None] * n
        self.used = [False] * n

    def __call__(self, vals, device) -> torch.Tensor:
        if self.host is None:
            self.host = torch.empty((self.n, len(vals)), dtype=torch.float32).pin_memory()
            self.host_np = self.host.numpy()
            self.events = [torch.cuda.Event() for _ in range(self.n)]
        k, self.k = self.k, (self.k + 1) % self.n
        if self.used[k]:
            self.events[k].synchronize()
        self.host_np[k, :] = vals  # (float64 -> float32 rounding, as torch.tensor(vals, float32))
        out = torch.empty(len(vals), dtype=torch.float32, device=device)
        out.copy_(self.host[k], non_blocking=True)
        self.events[k].record(torch.cuda.current_stream(device))
        self.used[k] = True
        return out


_ARGS_RING = _ArgsRing()


def _check_dense_moments(p: torch.Tensor, st: dict) -> None:
    """A dense update reads and writes p.numel() moment elements: a moment left in a sharded (rows
    or columns) layout would be overrun, so refuse it instead of launching."""
    for k in ("exp_avg", "exp_avg_sq"):
        if st[k].shape != p.shape:
            raise RuntimeError(f"AdamW: {k} has shape {tuple(st[k].shape)} but the parameter is {tuple(p.shape)} "
                               "(sharded table moments; release_tables() gathers them before a dense step)")


def _host_adam_args(lr, b1, b2, eps, wd, step, device) -> torch.Tensor:
    """The per-step scalars of make_adam (csrc/common.hpp) formed in Python doubles, rounded to
    fp32 once, as a TT_ADAM_ARGS_BYTES device buffer (staged through _ArgsRing: no host sync)."""
    vals = [1.0 - lr * wd, 1.0 - b1, b2, 1.0 - b2, lr / (1.0 - b1 ** step), math.sqrt(1.0 - b2 ** step), eps, 0.0]
    if torch.cuda.is_current_stream_capturing():
        raise RuntimeError("host AdamW scalars cannot be staged inside a graph capture")
    return _ARGS_RING(vals, torch.device(device))


def _merge_parts(parts, table: torch.Tensor, padding_idx):
    """One (ids, d_pooled, denom, plan) for every bag call on the table this step (a single call
    in the fused TwoTower path; separate tower calls are concatenated and re-planned)."""
    group = getattr(getattr(table, "_tt_deferred", None), "gather_group", None)
    if len(parts) == 1:
        ids, dp, den, plan = parts[0]
        if plan is None and table.is_cuda:
            plan = ops.BagPlan(ids, table.shape[0], table.shape[1], padding_idx, gather_group=group)
        return ids, dp, den, plan
    L = max(p[0].shape[1] for p in parts)
    ids = torch.cat([F.pad(p[0].to(torch.int64), (0, L - p[0].shape[1])) for p in parts], 0)
    if any(p[2] is None for p in parts):  # some parts arrived pre-divided: divide the others here
        dp = torch.cat([p[1] if p[2] is None else p[1] / p[2].unsqueeze(1) for p in parts], 0)
        den = None
    else:
        dp = torch.cat([p[1] for p in parts], 0)
        den = torch.cat([p[2] for p in parts], 0)
    return ids, dp, den, ops.BagPlan(ids, table.shape[0], table.shape[1], padding_idx, gather_group=group)
