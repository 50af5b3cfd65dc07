"""Data parallelism for the two-tower step: one process per GPU, torch.distributed over RCCL
(backend "nccl" on ROCm) across xGMI; gloo for the CPU tests of the same logic.

The reference has no distributed code.  This module adds exactly the exchanges
the step needs:
  * in-batch negatives: the candidate embeddings of every rank are all-gathered (rank-major),
    rank r's labels are offset by r * local_M, and the gather's backward reduce-scatters the
    candidate gradients back to their owners;
  * gradient sync: the loss is pre-scaled by 1/world so one SUM all-reduce per bucket yields the
    global-batch mean gradient for the small tower parameters;
  * embedding tables (ShardedRows, driven by optim.AdamW): the dense table gradient is
    reduce-scattered by row range, each rank runs AdamW on its own 1/world of the rows (and keeps
    only that shard's moments), and the updated rows are all-gathered in place -- the same bytes
    on the links as an all-reduce, 1/world of the optimizer's 24 B/param HBM traffic per rank.
    The rows go in chunks with interleaved ownership, so chunk c's exchange runs on a
    communication stream while the gradient of chunk c + 1 is formed.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

# HIP-graph capture of the N-rank step (train_step.TrainStep): ProcessGroupNCCL's event cache hands
# the end events of finished eager collectives to the collectives recorded during a capture while
# its watchdog thread may still query them, and the query of an event last recorded in a capturing
# stream fails ("operation not permitted on an event last recorded in a capturing stream": one run
# of tests/_dp_graph_check.py, round 3).  Fresh events per collective; the variable is read when a
# process group is created, so it is set here, before the caller creates one.  That protects only
# groups created after this import with the variable left alone: capture_blocker() tells the
# others apart, and TrainStep then stays eager instead of capturing.
_EVENT_CACHE_VAR = "TORCH_NCCL_CUDA_EVENT_CACHE"
# what held when this module was imported, read BEFORE the default below is applied: the caller's
# own value (None: unset), and whether a process group already existed (its ProcessGroupNCCL then
# read the variable at its creation, before the default could apply: an unset variable meant the
# cache was on)
_AT_IMPORT = {"event_cache": os.environ.get(_EVENT_CACHE_VAR),
              "group_existed": dist.is_available() and dist.is_initialized()}
os.environ.setdefault(_EVENT_CACHE_VAR, "0")


def _backend_kind(group=None) -> str:
    """"nccl", "gloo" or "other" for `group`'s backend; a mixed device:backend string
    ('cuda:nccl,cpu:gloo') counts as nccl, since its GPU collectives are ProcessGroupNCCL's."""
    b = str(dist.get_backend(group)).lower()
    if "nccl" in b:
        return "nccl"
    return "gloo" if "gloo" in b else "other"


def capture_blocker(group=None) -> str | None:
    """Why the N-rank step must not be captured in a HIP graph on `group`, or None if it may be.

    ProcessGroupNCCL with its CUDA event cache on hands the end events of eager collectives to
    collectives recorded during a capture, and its watchdog thread then queries an event last
    recorded in a capturing stream: an uncatchable abort (std::terminate in the watchdog).  The
    cache is off only for a group created while TORCH_NCCL_CUDA_EVENT_CACHE=0; this module sets
    that default at import, so a group created before the import without the caller having set
    the variable to '0', or any group while the variable is anything else, is refused here.  gloo
    groups are not captured at all (their collectives stage through host memory)."""
    if not (dist.is_available() and dist.is_initialized()):
        return None
    kind = _backend_kind(group)
    if kind == "gloo":
        return "gloo collectives cannot be captured in a HIP graph"
    if kind != "nccl":
        return None
    if _AT_IMPORT["group_existed"]:
        if _AT_IMPORT["event_cache"] != "0":
            return (f"the process group was created before twotower_amd.distributed was imported, with "
                    f"{_EVENT_CACHE_VAR}={_AT_IMPORT['event_cache']!r} (not '0': ProcessGroupNCCL's event cache "
                    f"aborts the watchdog under graph capture)")
        return None
    if os.environ.get(_EVENT_CACHE_VAR) != "0":
        return (f"{_EVENT_CACHE_VAR} is {os.environ.get(_EVENT_CACHE_VAR)!r}, not '0' (ProcessGroupNCCL's event "
                f"cache aborts the watchdog under graph capture)")
    return None


def is_active(group=None) -> bool:
    """Data-parallel exchanges on: more than one rank, or TT_DIST_FORCE=1 with any initialised
    group (a one-rank rehearsal of every collective of the N-rank step, e.g. RCCL under HIP-graph
    capture on a one-GPU box: bench.py --force-dist)."""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return dist.get_world_size(group) > 1 or os.environ.get("TT_DIST_FORCE") == "1"


def table_sync_mode(requested: str, group=None, E: int | None = None) -> str:
    """How an embedding table's gradient crosses ranks:
      "local"  -- one rank (no exchange);
      "gather" -- all-gather the factored gradient (ids in the forward, d_pooled/denom after the
                  backward: ~31 MB per rank at C3) and run the fused scatter + AdamW on every rank
                  over all ranks' entries (replicated table and moments, no parameter exchange);
      "shard"  -- reduce-scatter the dense table gradient by row range, AdamW on own rows,
                  all-gather the rows (2 x 205 MB x (N-1)/N per rank at C3);
      "owner"  -- all-gather the factored gradient as "gather" does, but each rank scatters and
                  updates only the rows it owns (shard's row partition and moment shards), then
                  the rows are all-gathered: (N-1) x 31 MB + 205 MB x (N-1)/N per rank at C3,
                  1/N of the update's HBM traffic, no dense gradient;
      "column" -- each rank owns E / N columns of every row (ColumnTable): the ids are all-gathered,
                  pooled and d_pooled column blocks exchanged all-to-all, no table row ever crosses
                  the links, 1/N of the update per rank (C5 at N = 8: ~0.26 GB per rank and step,
                  against 1.3-1.8 GB for owner / shard).
    "auto": gather up to 4 ranks, shard beyond.  Both keep a replicated, current table on every
    rank, so evaluation, search and state_dict() stay local (rank 0 alone may run them).
    "column" is the scaling choice (bench.py --gpus N takes it wherever column_ok) but opt-in:
    with a column-sharded table every forward that runs while the table is stale (after a step,
    until materialize() / state_dict()) is collective -- ids all-gather + pooled all-to-all --
    and state_dict() itself is collective (it materialises the slabs)."""
    if not is_active(group):
        return "local"
    if requested == "auto":
        world = dist.get_world_size(group)
        return "gather" if world <= 4 else "shard"
    if requested not in ("gather", "shard", "owner", "column"):
        raise ValueError(f"table_sync must be 'auto', 'gather', 'shard', 'owner' or 'column', got {requested!r}")
    return requested


def _is_gloo(group=None) -> bool:
    return _backend_kind(group) == "gloo"


def reduce_scatter_rows(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """out = rows [r*n, (r+1)*n) of the SUM over ranks of inp (n = out.shape[0])."""
    if _is_gloo(group):  # gloo has no reduce_scatter: all-reduce a copy and keep this rank's slab
        tmp = inp.clone()
        dist.all_reduce(tmp, op=dist.ReduceOp.SUM, group=group)
        r = dist.get_rank(group)
        out.copy_(tmp[r * out.shape[0]:(r + 1) * out.shape[0]])
        return
    dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=group)


def all_gather_rows(out: torch.Tensor, inp: torch.Tensor, group=None, async_op: bool = False):
    """out = cat over ranks of inp (rank-major); inp may be this rank's slab of out.  With
    async_op the work handle is returned (wait() before reading out), else None."""
    if _is_gloo(group):
        parts = list(out.chunk(dist.get_world_size(group)))
        return dist.all_gather(parts, inp.contiguous(), group=group, async_op=async_op)  # chunks are views of out
    return dist.all_gather_into_tensor(out, inp, group=group, async_op=async_op)


def shard_chunks(V: int, world: int) -> int:
    """Row chunks of the pipelined sharded-table exchange (TT_SHARD_CHUNKS, default 8): chunk c's
    reduce-scatter, AdamW and all-gather run on a communication stream while the gradient rows of
    chunk c + 1 are formed.  1 = one exchange after the whole gradient."""
    n = int(os.environ.get("TT_SHARD_CHUNKS", "8"))
    return max(1, min(n, V // max(1, world)))


def _agree(value: int, group, device, what: str) -> int:
    """`value`, checked equal on every rank of `group` (MIN and MAX all-reduced): a quantity that
    sizes collectives must not differ between ranks (a hang or corrupted rows otherwise)."""
    dev = device if dist.get_backend(group) != "gloo" else "cpu"
    t = torch.tensor([value, -value], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    lo, hi = int(t[0]), -int(t[1])
    if lo != hi:
        raise ValueError(f"ranks disagree on the {what}: {lo} .. {hi}")
    return value


class ShardedRows:
    """Row partition of a (V, E) table over the ranks of `group` for the sharded table optimizer.

    The rows are cut into NC chunks of world * R rows, and rank r owns rows
    [c*Cr + r*R, c*Cr + (r+1)*R) of every chunk c (Cr = world * R): interleaved ownership, so each
    chunk's reduce-scatter and all-gather move one contiguous slab per rank and can start as
    soon as that chunk's gradient rows exist (optim.AdamW pipelines them).  The parameter's
    storage is padded to Vp = NC * Cr rows (the padding rows stay zero and are never read by a
    lookup); this rank's moments are its Vs = NC * R own rows, chunk-major."""

    def __init__(self, weight: torch.Tensor, group=None, chunks: int | None = None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.V, self.E = weight.shape
        self.NC = _agree(chunks or shard_chunks(self.V, self.world), group, weight.device,
                         "row chunks of the sharded table (TT_SHARD_CHUNKS)")
        self.R = -(-self.V // (self.NC * self.world))
        self.Cr = self.R * self.world
        self.Vp = self.NC * self.Cr
        self.Vs = self.NC * self.R
        base = weight.data
        room = base.untyped_storage().nbytes() // base.element_size() - base.storage_offset()
        if not base.is_contiguous() or room < self.Vp * self.E:
            padded = torch.zeros(self.Vp, self.E, dtype=base.dtype, device=base.device)
            padded[:self.V].copy_(base)
            weight.data = padded[:self.V]
        self.weight = weight
        self._bufs = None
        self._comm = None

    def storage(self) -> torch.Tensor:
        """The (Vp, E) tensor the parameter is a view of."""
        w = self.weight.data
        return w if self.Vp == self.V else torch.as_strided(w, (self.Vp, self.E), (self.E, 1))

    def chunk(self, c: int) -> tuple[int, int]:
        """Rows [lo, hi) of chunk c in the (Vp, E) layout."""
        return c * self.Cr, (c + 1) * self.Cr

    def own(self, t: torch.Tensor, c: int) -> torch.Tensor:
        """This rank's slab of chunk c of a (Vp, E) tensor (a view)."""
        lo = c * self.Cr + self.rank * self.R
        return t[lo:lo + self.R]

    def shard_chunk(self, t: torch.Tensor, c: int) -> torch.Tensor:
        """Chunk c of a (Vs, E) per-rank tensor (a view)."""
        return t[c * self.R:(c + 1) * self.R]

    def rows(self, t: torch.Tensor) -> torch.Tensor:
        """This rank's rows of a (Vp, E) tensor as a (Vs, E) tensor, chunk-major (a view for one
        chunk, a copy otherwise)."""
        if self.NC == 1:
            return self.own(t, 0)
        return t.view(self.NC, self.world, self.R, -1)[:, self.rank].reshape(self.Vs, -1)

    def gather_full(self, shard: torch.Tensor) -> torch.Tensor:
        """The (Vp, E) tensor whose own rows on every rank are that rank's (Vs, E) shard."""
        buf = shard.new_empty(self.world * self.Vs, shard.shape[1])
        all_gather_rows(buf, shard.contiguous(), self.group)
        return buf.view(self.world, self.NC, self.R, -1).transpose(0, 1).reshape(self.Vp, -1)

    def new_grad_buffer(self) -> torch.Tensor:
        g = torch.empty(self.Vp, self.E, dtype=torch.float32, device=self.weight.device)
        if self.Vp != self.V:
            g[self.V:].zero_()
        return g

    def step_buffers(self) -> tuple[torch.Tensor, torch.Tensor]:
        """Persistent (gradient (Vp, E), reduced shard (Vs, E)) buffers of the pipelined update
        (fixed addresses, so the step can be captured in a HIP graph)."""
        if self._bufs is None:
            self._bufs = (self.new_grad_buffer(),
                          torch.empty(self.Vs, self.E, dtype=torch.float32, device=self.weight.device))
        return self._bufs

    def comm_stream(self) -> torch.cuda.Stream:
        if self._comm is None:
            self._comm = torch.cuda.Stream(device=self.weight.device)
        return self._comm

    def reduce_scatter(self, gbuf: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        shard = torch.empty(self.Vs, self.E, dtype=gbuf.dtype, device=gbuf.device) if out is None else out
        for c in range(self.NC):
            lo, hi = self.chunk(c)
            reduce_scatter_rows(self.shard_chunk(shard, c), gbuf[lo:hi], self.group)
        return shard

    def all_gather_params(self) -> None:
        st = self.storage()
        for c in range(self.NC):
            lo, hi = self.chunk(c)
            all_gather_rows(st[lo:hi], self.own(st, c), self.group)


def all_to_all_rows(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """Equal-split all-to-all over rows: block s of `out` (rows [s n, (s + 1) n), n = rows / world)
    = block r of rank s's `inp`, r = this rank."""
    world = dist.get_world_size(group)
    if _is_gloo(group):  # no gloo all-to-all on GPU tensors: all-gather the send buffers, keep our blocks
        full = inp.new_empty((world,) + tuple(inp.shape))
        all_gather_rows(full.view((world * inp.shape[0],) + tuple(inp.shape[1:])), inp.contiguous(), group)
        n = inp.shape[0] // world
        r = dist.get_rank(group)
        out.copy_(full[:, r * n:(r + 1) * n].reshape(out.shape))
        return
    dist.all_to_all_single(out, inp.contiguous(), group=group)


COLUMN_WIDTHS = (32, 64, 128, 256)  # slab widths El the column kernels take (tt_bag_col_reduce)


def column_ok(E: int, world: int) -> bool:
    """A (V, E) table can be column-sharded over `world` ranks."""
    return world >= 1 and E % world == 0 and E // world in COLUMN_WIDTHS


class ColumnTable:
    """Column partition of a (V, E) embedding table over the ranks of `group` (table_sync
    "column"): rank r owns columns [r El, (r + 1) El) of EVERY row, El = E / world, as a compact
    (V, El) fp32 slab with its AdamW moments.  Nothing of the table crosses the links:
      * forward: every rank's ids are all-gathered, each rank pools ITS columns for every rank's
        sequences (tt_bag_mean_fwd_cols over the slab, El wide, the full-width sum order) and the pooled column blocks are
        exchanged all-to-all, so each rank gets its own sequences' whole pooled rows;
      * backward: d_pooled / denom is cut into column blocks and exchanged all-to-all, and each rank
        forms the gradient of its slab from every rank's tokens (the per-rank sort plans,
        all-gathered during the forward, merged in rank order: tt_bag_col_reduce) fused with AdamW
        on its slab -- the dense AdamW of train.py:139 over every element, exactly once, 1/world of
        the table's optimizer traffic per rank.
    The parameter tensor (V, E) is kept for the model's API (state_dict keys, shapes) but goes
    stale after the first update: materialize() all-gathers the slabs into it (a collective: every
    rank calls it), and the owning nn.Embedding does so before state_dict() (a pre-hook); a
    load_state_dict() into the module reloads the slab from the loaded weight."""

    def __init__(self, weight: torch.Tensor, group=None, module: torch.nn.Module | None = None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.V, self.E = weight.shape
        if not column_ok(self.E, self.world):
            raise ValueError(f"table_sync 'column' needs E / world in {COLUMN_WIDTHS} (E {self.E}, world {self.world})")
        self.El = self.E // self.world
        self.c0 = self.rank * self.El
        self.weight = weight
        self.slab = weight.detach()[:, self.c0:self.c0 + self.El].contiguous().clone()
        self.stale = False
        if module is not None:
            module.register_state_dict_pre_hook(lambda *_a, **_k: self.materialize())
            module.register_load_state_dict_post_hook(lambda *_a, **_k: self.load_from_weight())

    def gather_cols(self, t: torch.Tensor) -> torch.Tensor:
        """(V, E) tensor whose column block r is rank r's (V, El) `t` (an all-gather)."""
        buf = t.new_empty(self.world * self.V, self.El)
        all_gather_rows(buf, t.contiguous(), self.group)
        return buf.view(self.world, self.V, self.El).permute(1, 0, 2).reshape(self.V, self.E)

    def own_cols(self, full: torch.Tensor) -> torch.Tensor:
        """This rank's (V, El) columns of a (V, E) tensor (a copy)."""
        return full[:, self.c0:self.c0 + self.El].contiguous()

    @torch.no_grad()
    def materialize(self) -> None:
        """Write every rank's slab into the (V, E) parameter (collective)."""
        if self.stale:
            self.weight.data.copy_(self.gather_cols(self.slab))
            self.stale = False

    @torch.no_grad()
    def load_from_weight(self) -> None:
        self.slab.copy_(self.weight.data[:, self.c0:self.c0 + self.El])
        self.stale = False


class AllGatherRows(torch.autograd.Function):
    """out = cat over ranks of x (rank-major); backward = reduce_scatter(SUM) of the gradient."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        world = dist.get_world_size(group)
        x = x.contiguous()
        out = x.new_empty((world * x.shape[0],) + tuple(x.shape[1:]))
        all_gather_rows(out, x, group)
        return out

    @staticmethod
    def backward(ctx, g):
        world = dist.get_world_size(ctx.group)
        g = g.contiguous()
        out = g.new_empty((g.shape[0] // world,) + tuple(g.shape[1:]))
        reduce_scatter_rows(out, g, ctx.group)
        return out, None


def gather_candidates(d: torch.Tensor, group=None) -> tuple[torch.Tensor, int]:
    """All ranks' candidate rows and this rank's label offset (its first candidate row)."""
    if not is_active(group):
        return d, 0
    return AllGatherRows.apply(d, group), dist.get_rank(group) * d.shape[0]


class GradSync:
    """Sum-all-reduce of every gradient after backward.  Small parameters travel in one flat
    bucket; large ones (the embedding table) are reduced in place.  With the loss pre-scaled
    by 1/world the sums are the global-batch mean gradients.

    Two ways to run it:
      * ``sync()`` -- after backward, before the optimizer (any optimizer);
      * ``launch(side)`` -- called by optim.AdamW inside ``step()`` once it has issued the table
        exchange and launched the fused table update: the all-reduce runs on a communication
        stream that waits only for the gradients' producers (the backward on the current stream
        and the "wgrad" side stream of ops.TowerHead), so it overlaps the table update, and its
        completion event joins the optimizer's SideGrads, which the dense AdamW waits for.
        The table's collectives are issued before it, so they are not queued behind the tower
        gradients on the communicator."""

    def __init__(self, params, group=None, bucket_cap: int = 1 << 22):
        self.group = group
        self.params = [p for p in params if p.requires_grad]
        self.bucket_cap = bucket_cap
        self._streams: dict = {}

    @property
    def world(self) -> int:
        return dist.get_world_size(self.group) if is_active(self.group) else 1

    def loss_scale(self) -> float:
        return 1.0 / self.world

    def _split(self):
        small = [p for p in self.params if p.grad is not None and p.numel() <= self.bucket_cap]
        large = [p for p in self.params if p.grad is not None and p.numel() > self.bucket_cap]
        return small, large

    def _reduce(self, small, large) -> None:
        # synchronous collectives: they queue on the communicator's stream behind each other
        # either way, and an async_op collective waited on a forked stream crashes HIP graph
        # capture at its end on this image (tools/repro/capture_probe.py side_async_ar: segfault in
        # hipStreamEndCapture; the same all-reduce without async_op captures and replays)
        if small:
            flat = torch.cat([p.grad.reshape(-1) for p in small])
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
            off = 0
            for p in small:
                n = p.numel()
                p.grad.copy_(flat[off:off + n].view_as(p.grad))
                off += n
        for p in large:
            dist.all_reduce(p.grad, op=dist.ReduceOp.SUM, group=self.group)

    def sync(self) -> None:
        if not is_active(self.group):
            return
        from ._lib import join_side_grads

        join_side_grads(self.params)  # gradients computed on a side stream (ops.TowerHead)
        self._reduce(*self._split())

    def launch(self, side, after=None) -> None:
        """The all-reduce on a communication stream; its completion joins ``side`` (a
        _lib.SideGrads the caller joins before reading the gradients).  ``after``: an event the
        caller recorded on the current stream where the gradients are complete (optim.AdamW: the
        end of backward, before it queues the table update); without it the communication stream
        waits for everything queued so far.  CPU tensors (gloo tests) or no side object: the plain
        synchronous ``sync()``."""
        if not is_active(self.group):
            return
        small, large = self._split()
        grads = [p.grad for p in small + large]
        if side is None or not grads or not all(g.is_cuda for g in grads):
            self.sync()
            return
        dev = grads[0].device
        comm = self._streams.get(dev)
        if comm is None:
            comm = self._streams[dev] = torch.cuda.Stream(device=dev)
        if after is not None:  # gradients written by the main-stream backward
            comm.wait_event(after)
        else:
            comm.wait_stream(torch.cuda.current_stream(dev))
        for ev in side.events:  # ... and by the wgrad side stream
            comm.wait_event(ev)
        with torch.cuda.stream(comm):
            side.run_finals()  # e.g. the weight gradients' slab sums, before they are reduced
            self._reduce(small, large)
            done = torch.cuda.Event()
            done.record(comm)
        for g in grads:
            g.record_stream(comm)
        side.events.append(done)
