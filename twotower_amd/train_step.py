"""One training step of the two-tower model, the body of the reference's hot loop
(twotower/train.py:103-139: forward :120-122, loss :133, zero_grad/backward/step :137-139),
with optional data parallelism.  Returns the loss as a device tensor (no host sync; the
reference's per-step .item() monitors at :144-154 are left to the caller).

``graph=True`` captures the whole step (forward, loss, backward, optimizer) in one HIP graph
after ``eager_steps`` ordinary steps and replays it for every later batch of the same shape:
the step's ~40 kernel launches then cost one graph launch, and the GPU no longer idles while
Python issues short kernels.  Each call is still exactly one training step on its own batch
(the batch is copied into the graph's static input buffers first).  Needs a capturable
optimizer (optim.AdamW(capturable=True)); a new input shape is captured anew.
"""
from __future__ import annotations

import contextlib
import os

import torch

from . import ops
from .distributed import GradSync, capture_blocker, is_active
from .losses import scorer_prep_dtype


class TrainStep:
    def __init__(self, model: torch.nn.Module, loss_fn, optimizer: torch.optim.Optimizer, group=None,
                 graph: bool = False, eager_steps: int = 2):
        self.model = model
        self.loss_fn = loss_fn
        self.optimizer = optimizer
        self.group = group
        self.sync = GradSync(model.parameters(), group=group) if is_active(group) else None
        # an optimizer that launches the gradient all-reduce itself, after its own table exchange
        # (optim.AdamW): the all-reduce then overlaps the table update
        # (set on the optimizer only for the duration of this step's optimizer.step(): a plain loop
        # that calls GradSync.sync() itself must not see a second all-reduce)
        self._sync_in_step = self.sync is not None and hasattr(optimizer, "_grad_sync")
        # a single-device bf16 in-batch loss: the tied towers' head prepares its operands
        # (TT_SCORER_PREP=0: the loss's own prep pass, for comparison)
        # Opened only around this step's own forward (_scorer_prep_open): set on the model for
        # good, every later forward (eval, export, another loss) would prep operands no one reads.
        dt = scorer_prep_dtype(loss_fn)
        self._scorer_prep = (dt if dt is not None and hasattr(model, "scorer_prep") and not is_active(group)
                             and os.environ.get("TT_SCORER_PREP", "1") != "0" else None)
        # The in-batch loss may leave its mean to the backward's combine launch only when the
        # tensor loss_fn returns IS that loss (the bare registry partial): a wrapper (a scaled or
        # summed loss, a .item() log inside loss_fn) reads the value before the backward forms it.
        self._defer_mean = dt is not None
        self.graph = graph
        if graph and not all(g.get("capturable", False) for g in optimizer.param_groups):
            raise ValueError("TrainStep(graph=True) needs an optimizer built with capturable=True")
        self._eager_left = max(1, int(eager_steps))  # >= 1: lazy library/workspace set-up happens eagerly
        self._graphs: dict[tuple, tuple] = {}
        self._seed: dict[torch.device, torch.Tensor] = {}  # d(loss) seed of backward, kept on device

    def eager(self, queries: torch.Tensor, positive_docs: torch.Tensor,
              negative_docs: torch.Tensor | None = None) -> torch.Tensor:
        """One step.  negative_docs None: a (query, positive) pair step -- model(q, p), loss_fn(q, p)
        (e.g. the in-batch loss over the positives alone)."""
        # forward, backward and step back to back: the optimizer may take gradients computed on
        # a side stream and join them itself (_lib.SideGrads)
        side = getattr(self.optimizer, "_side_grads", None)
        if side is not None:
            side.join()
            side.active = True
        try:
            defer = ops.deferred_loss_mean() if self._defer_mean else contextlib.nullcontext()
            with defer, self._scorer_prep_open():  # the loss is read after the backward below
                ins = (queries, positive_docs) if negative_docs is None else (queries, positive_docs, negative_docs)
                loss = self.loss_fn(*self.model(*ins))
            self.optimizer.zero_grad(set_to_none=True)
            # backward seeded with the (1/world pre-scaled) unit gradient from a resident tensor:
            # no fill / scale kernels per step
            seed = self._seed.get(loss.device)
            if seed is None:
                scale = self.sync.loss_scale() if self.sync is not None else 1.0
                seed = self._seed[loss.device] = torch.full((), scale, dtype=loss.dtype, device=loss.device)
            # every rank seeds its loss alike (1/world); the heads' outputs reach only the loss
            with ops.uniform_loss_seed(), ops.fused_head_backward():
                loss.backward(seed)
            if self.sync is not None and not self._sync_in_step:
                self.sync.sync()
            if self._sync_in_step:  # the optimizer launches the all-reduce inside this step only
                self.optimizer._grad_sync = self.sync
            self.optimizer.step()
        finally:
            if self._sync_in_step:
                self.optimizer._grad_sync = None
            if side is not None:
                side.active = False
                side.join()  # no-op after the optimizer's own join
        return loss.detach()

    @contextlib.contextmanager
    def _scorer_prep_open(self):
        if self._scorer_prep is None:
            yield
            return
        prev = self.model.scorer_prep
        self.model.scorer_prep = self._scorer_prep
        try:
            yield
        finally:
            self.model.scorer_prep = prev

    def __call__(self, queries: torch.Tensor, positive_docs: torch.Tensor,
                 negative_docs: torch.Tensor | None = None) -> torch.Tensor:
        if not self.graph:
            return self.eager(queries, positive_docs, negative_docs)
        inputs = (queries, positive_docs) if negative_docs is None else (queries, positive_docs, negative_docs)
        key = tuple((tuple(t.shape), t.dtype, t.device) for t in inputs)
        hit = self._graphs.get(key)
        if hit is None:
            if self._eager_left > 0:
                self._eager_left -= 1
                return self.eager(*inputs)
            why = capture_blocker(self.group) if is_active(self.group) else None
            err = fatal = None
            if why is None:
                try:
                    hit = self._capture(inputs)
                except RuntimeError as e:  # e.g. a collective this backend cannot capture
                    if _is_capture_error(e):
                        err = e
                    else:
                        fatal = e  # a real error of the step itself: not hidden behind a fallback
            # every rank replays, or none does: a rank whose capture failed steps eagerly, and its
            # collectives must not meet graph-replayed ones on the other ranks.  A rank whose step
            # raised joins the agreement too (code -1) before it re-raises, so its peers fail at
            # once instead of waiting in their next collective until the backend's timeout.
            code = -1 if fatal is not None else (1 if why is None and err is None else 0)
            if is_active(self.group):
                code = _all_ranks_min(code, self.group, inputs[0].device)
            if code < 0:
                self._discard_partial_step()
                if fatal is not None:
                    raise fatal
                raise RuntimeError("TrainStep: another rank's step raised while its HIP graph was captured")
            if code == 0:
                import warnings

                self._discard_partial_step()
                reason = why or (f"HIP graph capture failed ({err})" if err is not None
                                 else "another rank's HIP graph capture failed")
                warnings.warn(f"TrainStep: {reason}; running the step eagerly")
                self.graph = False
                return self.eager(*inputs)
            self._graphs[key] = hit
        graph, static_all, static_loss = hit
        if all(t.shape[1:] == inputs[0].shape[1:] and t.dtype == inputs[0].dtype for t in inputs):
            if all(t.device == static_all.device and t.is_contiguous() for t in inputs) and len(inputs) <= 8:
                ops.pack_blocks(inputs, static_all)  # one launch into the packed static buffer
            else:
                torch.cat(inputs, 0, out=static_all)
        else:
            for dst, src in zip(_views(static_all, inputs), inputs):
                dst.copy_(src)
        graph.replay()
        return static_loss

    def release(self) -> None:
        """Drop the captured graphs (and the static buffers they own).  Call before tearing down the
        process group: a replayable graph keeps the RCCL resources of the collectives it captured
        (the point-to-point sends and receives of an all-to-all among them) registered with the
        communicator, whose destruction would otherwise wait for them."""
        torch.cuda.synchronize()
        self._graphs.clear()
        import gc

        gc.collect()
        torch.cuda.synchronize()

    def _discard_partial_step(self) -> None:
        """Forget what a failed capture queued for the optimizer: the factored table gradients the
        bag backward handed over and the side-stream gradient events (none of that ran)."""
        for g in self.optimizer.param_groups:
            for p in g["params"]:
                deferred = getattr(p, "_tt_deferred", None)
                if deferred is not None:
                    deferred.parts.clear()
        side = getattr(self.optimizer, "_side_grads", None)
        if side is not None:
            side.reset()
        self.optimizer.zero_grad(set_to_none=True)

    def _capture(self, inputs):
        # the static inputs are consecutive row blocks of one buffer, so the fused TwoTower
        # forward uses them in place (no concatenation inside the step)
        static_all = _packed_like(inputs)
        static_in = tuple(_views(static_all, inputs))
        for dst, src in zip(static_in, inputs):
            dst.copy_(src)
        graph = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        # thread-local capture mode: a process group's watchdog thread polls the events of the
        # collectives issued before the capture (hipEventQuery); under the default global mode
        # that query is refused while this thread captures and the watchdog aborts the process
        # (seen once in the one-rank RCCL graph test: "operation not permitted when stream is
        # capturing" from the ProcessGroupNCCL watchdog).  Calls made by this thread are checked
        # as before.
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            static_loss = self.eager(*static_in)
        return graph, static_all, static_loss


# messages of errors raised because a call is refused inside stream capture (HIP's and CUDA's
# error names and texts, torch's own capture guards), matched as whole phrases: a broad substring
# ("captur", "not permitted") would also hide unrelated errors behind the eager fallback
_CAPTURE_ERRORS = (
    "hiperrorstreamcapture",  # hipErrorStreamCaptureUnsupported / Invalidated / Unjoined / Isolation ...
    "cudaerrorstreamcapture",
    "operation not permitted when stream is capturing",
    "operation not permitted on an event last recorded in a capturing stream",
    "operation would make the legacy stream depend on a capturing blocking stream",
    "during cuda graph capture",
    "during hip graph capture",
    "while a stream is capturing",
    "hiperrorcapturedevent",  # an event recorded in a capturing stream, queried / synchronised
    "cudaerrorcapturedevent",
    "stream is capturing",
    "stream capture",  # "... not allowed during stream capture", "stream capture invalidated" ...
    "graph capture",  # torch's / c10d's own guards ("... is not supported during (CUDA) graph capture")
    "is_current_stream_capturing",
    "capture_begin",
    "hipstreamcapturestatus",  # torch's capture_end assert when another call invalidated the capture
    "cudastreamcapturestatus",
)
# (the error-code enum names torch embeds in HIP/CUDA runtime errors cover the rest; messages seen
# on this stack from collectives refused under capture: tests/test_host_cpu.py::test_capture_error_messages)


def _is_capture_error(e: BaseException) -> bool:
    """An error raised because the step was being captured (a call HIP or a backend refuses inside
    stream capture), as opposed to an error of the step itself."""
    msg = str(e).lower()
    return any(k in msg for k in _CAPTURE_ERRORS)


def _all_ranks_min(code: int, group, device) -> int:
    """MIN of `code` over the ranks of `group` (an all-reduce outside any capture)."""
    import torch.distributed as dist

    t = torch.tensor([int(code)], dtype=torch.int32,
                     device=device if dist.get_backend(group) != "gloo" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return int(t.item())


def _packed_like(inputs):
    if all(t.shape[1:] == inputs[0].shape[1:] and t.dtype == inputs[0].dtype for t in inputs):
        return torch.empty((sum(t.shape[0] for t in inputs),) + tuple(inputs[0].shape[1:]), dtype=inputs[0].dtype,
                           device=inputs[0].device)
    return [t.clone() for t in inputs]


def _views(static_all, inputs):
    if isinstance(static_all, list):
        return static_all
    return torch.split(static_all, [t.shape[0] for t in inputs], 0)
