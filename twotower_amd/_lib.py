"""ctypes binding of libtwotower_amd.so (the C ABI declared in include/twotower_amd.h).

The product path has no fallback: if the shared library is missing, or a tensor is not on a
GPU, the call raises.  Torch only supplies device memory and the current HIP stream.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import re
import threading

import torch

# TT_LIB: another build of the library (measurement variants, tools/build_variants.sh)
LIB_PATH = os.environ.get("TT_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libtwotower_amd.so")
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "twotower_amd.h")

TT_IDS_I32, TT_IDS_I64 = 0, 1
TT_INBATCH_TAIL_ROWS, TT_INBATCH_MAX_PARTS = 64, 512  # twotower_amd.h
TT_F32, TT_BF16, TT_BF16_SPLIT = 0, 1, 2
TT_SCATTER_SORTED, TT_SCATTER_ATOMIC = 0, 1
TT_INBATCH_BWD_RECOMPUTE, TT_INBATCH_BWD_STORED = 0, 1

COMPUTE_DTYPES = {"fp32": TT_F32, "float32": TT_F32, "bf16": TT_BF16, "bfloat16": TT_BF16,
                  "bf16_split": TT_BF16_SPLIT}

_c_i64, _c_int, _c_f32, _c_sz, _vp = ctypes.c_int64, ctypes.c_int, ctypes.c_float, ctypes.c_size_t, ctypes.c_void_p
_c_f64 = ctypes.c_double

TT_ADAM_ARGS_BYTES = 32
TT_ADAM_MAX_TENSORS = 16
TT_ADAM_TICKET_WORDS = 16


class AdamSlot(ctypes.Structure):
    """tt_adam_slot"""
    _fields_ = [("step", _vp), ("args", _vp)]


class AdamwTensor(ctypes.Structure):
    """tt_adamw_tensor"""
    _fields_ = [("param", _vp), ("grad", _vp), ("exp_avg", _vp), ("exp_avg_sq", _vp), ("n", _c_i64), ("args", _vp)]


class AdamwGradParts(ctypes.Structure):
    """tt_adamw_grad_parts"""
    _fields_ = [("part", _vp), ("stride", _c_i64), ("slabs", _c_int)]


# name -> (restype, argtypes); must mirror include/twotower_amd.h
_SIGNATURES = {
    "tt_version": (_c_int, []),
    "tt_last_error": (ctypes.c_char_p, []),
    "tt_bag_mean_fwd": (_c_int, [_vp, _c_i64, _c_int, _vp, _c_int, _c_i64, _c_int, _c_i64, _vp, _vp, _vp]),
    "tt_bag_mean_fwd_cols": (_c_int, [_vp, _c_i64, _c_int, _c_int, _vp, _c_int, _c_i64, _c_int, _c_i64, _vp, _vp, _vp]),
    "tt_bag_mean_fwd_split": (_c_int, [_vp, _c_i64, _c_int, _vp, _c_int, _c_i64, _c_int, _c_i64, _vp, _vp, _vp, _vp,
                                       _c_int, _vp, _vp]),
    "tt_bag_mean_bwd_ws_size": (_c_sz, [_c_i64, _c_int, _c_i64, _c_int]),
    "tt_bag_mean_bwd": (_c_int, [_vp, _vp, _vp, _c_int, _c_i64, _c_int, _c_i64, _c_i64, _c_int, _c_i64, _vp, _c_int,
                                 _vp, _c_sz, _vp]),
    "tt_bag_mean_bwd_adamw": (_c_int, [_vp, _vp, _vp, _c_int, _c_i64, _c_int, _c_i64, _c_i64, _c_int, _c_i64, _vp,
                                       _vp, _vp, _c_f64, _c_f64, _c_f64, _c_f64, _c_f64, _c_i64, _vp, _c_sz, _vp]),
    "tt_bag_plan_ws_size": (_c_sz, [_c_i64, _c_int, _c_i64, _c_int]),
    "tt_bag_plan": (_c_int, [_vp, _c_int, _c_i64, _c_int, _c_i64, _c_i64, _c_int, _c_i64, _vp, _c_sz, _vp]),
    "tt_bag_plan_part": (_c_int, [_vp, _c_int, _c_i64, _c_int, _c_i64, _c_i64, _c_int, _c_i64, _vp, _c_sz, _c_int,
                                  _vp]),
    "tt_bag_plan_layout": (_c_int, [_c_i64, _c_int, _c_i64, _c_int, _vp]),
    "tt_bag_mean_bwd_planned": (_c_int, [_vp, _vp, _c_i64, _c_int, _c_i64, _c_int, _vp, _c_sz, _vp, _vp]),
    "tt_bag_mean_bwd_planned_prepare": (_c_int, [_vp, _vp, _c_i64, _c_int, _c_i64, _c_int, _vp, _c_sz, _vp]),
    "tt_bag_mean_bwd_planned_rows": (_c_int, [_vp, _vp, _c_i64, _c_int, _c_i64, _c_int, _vp, _c_sz, _c_i64, _c_i64,
                                              _vp, _vp]),
    "tt_bag_mean_bwd_adamw_planned": (_c_int, [_vp, _vp, _c_i64, _c_int, _c_i64, _c_int, _vp, _c_sz, _vp, _vp, _vp,
                                               _vp, _vp]),
    "tt_bag_mean_bwd_adamw_planned_rows": (_c_int, [_vp, _vp, _c_i64, _c_int, _c_i64, _c_int, _vp, _c_sz, _c_i64,
                                                    _c_i64, _vp, _vp, _vp, _vp, _vp]),
    "tt_bag_scale_rows": (_c_int, [_vp, _vp, _c_i64, _c_int, _vp, _vp]),
    "tt_bag_col_reduce": (_c_int, [_vp, _vp, _c_i64, _c_int, _c_i64, _vp, _c_i64, _c_int, _vp, _vp, _vp, _vp, _vp,
                                   _vp]),
    "tt_bag_col_reduce_ws_size": (_c_sz, [_c_i64, _c_int, _c_i64, _c_int]),
    "tt_bag_col_reduce_ex": (_c_int, [_vp, _vp, _c_i64, _c_int, _c_i64, _vp, _c_i64, _c_int, _vp, _vp, _vp, _vp,
                                      _vp, _vp, _c_sz, _vp]),
    "tt_adam_prepare": (_c_int, [ctypes.POINTER(AdamSlot), _c_int, _c_f64, _c_f64, _c_f64, _c_f64, _c_f64, _vp]),
    "tt_adam_prepare_ex": (_c_int, [ctypes.POINTER(AdamSlot), _c_int, _c_f64, _c_f64, _c_f64, _c_f64, _c_f64,
                                    _c_int, _c_int, _vp]),
    "tt_adamw_multi": (_c_int, [ctypes.POINTER(AdamwTensor), _c_int, _vp]),
    "tt_adamw_multi_ex": (_c_int, [ctypes.POINTER(AdamwTensor), ctypes.POINTER(AdamwGradParts), _c_int,
                                   ctypes.POINTER(AdamSlot), _c_int, _c_f64, _c_f64, _c_f64, _c_f64, _c_f64, _vp,
                                   _vp]),
    "tt_cosine_scores": (_c_int, [_vp, _c_i64, _vp, _c_i64, _c_int, _vp, _vp]),
    "tt_topk_rows": (_c_int, [_vp, _c_i64, _c_i64, _c_int, _vp, _vp, _vp]),
    "tt_topk_rows_ws_size": (_c_sz, [_c_i64, _c_i64, _c_int]),
    "tt_topk_rows_ex": (_c_int, [_vp, _c_i64, _c_i64, _c_int, _vp, _c_sz, _vp, _vp, _vp]),
    "tt_pack_blocks": (_c_int, [ctypes.POINTER(_vp), ctypes.POINTER(_c_i64), _c_int, _vp, _vp]),
    "tt_gather_rows_i32": (_c_int, [_vp, _c_i64, _c_i64, _vp, _c_i64, _c_int, _vp, _c_i64, _vp, _vp]),
    "tt_gather_rows_i32_ex": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _c_int, _vp, _c_i64, _c_int, _vp, _c_i64, _c_i64,
                                       _vp, _c_int, _vp]),
    "tt_ln_l2_fwd": (_c_int, [_vp, _c_i64, _c_int, _vp, _vp, _c_f32, _vp, _vp, _vp]),
    "tt_ln_l2_bwd": (_c_int, [_vp, _vp, _c_i64, _c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "tt_ln_l2_bwd_ws_size": (_c_sz, [_c_i64, _c_int]),
    "tt_ln_l2_bwd_ex": (_c_int, [_vp, _vp, _c_i64, _c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _c_sz, _vp]),
    "tt_head_planes_bytes": (_c_sz, [_c_int, _c_int]),
    "tt_head_split": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _vp]),
    "tt_head_split_ff": (_c_int, [_vp, _vp, _vp, _vp]),
    "tt_head_split_ff2": (_c_int, [_vp, _vp, _c_int, _c_int, _vp, _vp]),
    "tt_head_gemm_ws_size": (_c_sz, [_c_i64, _c_int]),
    "tt_head_relu_mask_bytes": (_c_sz, [_c_i64]),
    "tt_head_wgrad_ws_size": (_c_sz, [_c_i64, _c_int]),
    "tt_head_wgrad": (_c_int, [_vp, _vp, _c_i64, _c_int, _vp, _vp, _vp, _c_sz, _vp]),
    "tt_head_wgrad_ex_ws_size": (_c_sz, [_c_i64, _c_int, _c_int]),
    "tt_stamp": (_c_int, [_vp, _vp]),
    "tt_wall_clock_khz": (_c_int, [_c_int]),
    "tt_head_wgrad_ex": (_c_int, [_vp, _vp, _c_i64, _c_int, _c_int, _vp, _vp, _vp, _c_sz, _vp]),
    "tt_head_wgrad2_ws_size": (_c_sz, [_c_i64, _c_int]),
    "tt_head_wgrad2": (_c_int, [_vp, _vp, _vp, _vp, _c_i64, _c_int, _vp, _c_sz, _vp]),
    "tt_head_wgrad2_reduce": (_c_int, [_vp, _c_int, _vp, _vp, _vp, _vp, _vp]),
    "tt_head_wgrad2_parts": (_c_int, [_c_int, _c_int, ctypes.POINTER(_c_i64), ctypes.POINTER(_c_i64)]),
    "tt_head_gemm": (_c_int, [_vp, _c_i64, _c_i64, _c_int, _vp, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp, _c_sz,
                              _vp]),
    "tt_adamw": (_c_int, [_vp, _vp, _vp, _vp, _c_i64, _c_f64, _c_f64, _c_f64, _c_f64, _c_f64, _c_i64, _vp]),
    "tt_l2norm_fwd": (_c_int, [_vp, _c_i64, _c_int, _vp, _vp, _vp]),
    "tt_l2norm_bwd": (_c_int, [_vp, _vp, _vp, _c_i64, _c_int, _vp, _vp]),
    "tt_mean": (_c_int, [_vp, _c_i64, _vp, _vp]),
    "tt_colsum_ws_size": (_c_sz, [_c_i64, _c_int]),
    "tt_colsum": (_c_int, [_vp, _c_i64, _c_int, _vp, _vp, _c_sz, _vp]),
    "tt_relu_bwd": (_c_int, [_vp, _vp, _c_i64, _vp]),
    "tt_triplet_fwd": (_c_int, [_vp, _vp, _vp, _c_i64, _c_int, _c_f32, _vp, _vp, _vp]),
    "tt_triplet_bwd": (_c_int, [_vp, _vp, _vp, _c_i64, _c_int, _c_f32, _vp, _vp, _vp, _vp, _vp]),
    "tt_multi_neg_fwd": (_c_int, [_vp, _vp, _vp, _c_i64, _c_int, _c_int, _c_f32, _vp, _vp, _vp]),
    "tt_multi_neg_bwd": (_c_int, [_vp, _vp, _vp, _c_i64, _c_int, _c_int, _c_f32, _vp, _vp, _vp, _vp, _vp]),
    "tt_multi_neg_bwd_l2": (_c_int, [_vp, _c_i64, _c_int, _vp, _c_f32, _vp, _vp, _vp]),
    "tt_inbatch_set_backward": (_c_int, [_c_int]),
    "tt_inbatch_ws_size": (_c_sz, [_c_i64, _c_i64, _c_int, _c_int]),
    "tt_inbatch_fwd": (_c_int, [_vp, _vp, _c_i64, _c_i64, _c_int, _c_int, _c_f32, _c_i64, _c_int, _vp, _vp, _vp, _vp,
                                _vp, _c_sz, _vp]),
    "tt_inbatch_bwd": (_c_int, [_vp, _vp, _c_i64, _c_i64, _c_int, _c_int, _c_f32, _c_i64, _vp, _vp, _vp, _c_f32, _vp,
                                _vp, _vp, _vp, _vp, _c_sz, _vp]),
    "tt_inbatch_bwd_l2": (_c_int, [_vp, _c_i64, _c_i64, _c_int, _c_int, _c_f32, _c_i64, _vp, _vp, _vp, _c_f32, _vp,
                                   _vp, _vp, _vp, _vp, _c_sz, _vp]),
    "tt_inbatch_l2_prep": (_c_int, [_vp, _c_i64, _c_i64, _c_int, _c_int, _vp, _vp, _c_sz, _vp]),
    "tt_inbatch_fwd_prepped": (_c_int, [_vp, _vp, _c_i64, _c_i64, _c_int, _c_int, _c_f32, _c_i64, _c_int, _vp, _vp,
                                        _vp, _vp, _vp, _c_sz, _vp]),
    "tt_inbatch_prep_rows": (_c_int, [_vp, _c_i64, _c_int, _vp, _vp, _vp, _vp]),
    "tt_inbatch_ex_ws_size": (_c_sz, [_c_i64, _c_i64, _c_i64, _c_i64, _c_int, _c_int]),
    "tt_inbatch_fwd_ex": (_c_int, [_vp, _vp, _c_i64, _vp, _vp, _c_int, _c_i64, _c_int, _c_int, _c_f32, _c_i64, _c_int,
                                   _vp, _vp, _vp, _vp, _vp, _vp, _c_sz, _vp]),
    "tt_inbatch_fwd_ex_local": (_c_int, [_vp, _vp, _c_i64, _vp, _vp, _c_int, _c_i64, _c_i64, _c_i64, _c_int, _c_int,
                                         _c_f32, _vp, _c_sz, _vp]),
    "tt_inbatch_fwd_ex_remote": (_c_int, [_vp, _vp, _c_i64, _vp, _vp, _c_int, _vp, _c_int, _c_i64, _c_i64, _c_i64,
                                          _c_int, _c_int, _c_f32, _c_int, _vp, _vp, _vp, _vp, _vp, _vp, _c_sz, _vp]),
    "tt_inbatch_bwd_ex": (_c_int, [_vp, _vp, _c_i64, _c_i64, _vp, _c_i64, _c_i64, _c_i64, _c_int, _c_int, _c_f32, _vp,
                                   _vp, _c_f32, _vp, _vp, _vp, _c_sz, _vp]),
}

_lock = threading.Lock()
_lib = None


def header_symbols(path: str = HEADER_PATH) -> list[str]:
    """Every function the public header declares (used by the ABI export test)."""
    text = open(path).read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t|const char\*)\s+(tt_\w+)\s*\(", text, flags=re.M)))


def side_stream(device: torch.device, role: str = "plan") -> torch.cuda.Stream:
    """A per-device auxiliary stream.  role "plan": id-only work that runs beside the forward
    (the bag backward's sort plan); role "wgrad": the tower weight gradients, which run beside
    the fused table update (see SideGrads)."""
    dev = torch.device(device)
    key = (dev.index if dev.index is not None else torch.cuda.current_device(), role)
    st = _SIDE.get(key)
    if st is None:
        # (normal priority: a high-priority plan stream made the C3 step 1.42 vs 0.82 ms, round 4,
        # profiles/r04e_plan_priority_ab.txt)
        st = _SIDE[key] = torch.cuda.Stream(device=key[0])
    return st


_SIDE: dict[tuple, torch.cuda.Stream] = {}


class SideGrads:
    """Gradients produced on a side stream, joined by whoever consumes them.

    An optimizer that can order its own work (optim.AdamW) attaches one SideGrads to each of its
    dense parameters (``param._tt_side_grads``).  While it is ``active`` -- set by a caller that
    runs backward and the optimizer step back to back (train_step.TrainStep), so no one reads
    ``.grad`` in between -- a backward that finds it there computes that parameter's gradient
    on the "wgrad" side stream and registers the completion event; the optimizer launches work
    that does not read those gradients first (the fused table scatter + AdamW) and calls
    ``join()`` on the current stream before reading them.  Otherwise the backward computes on
    the current stream as usual."""

    def __init__(self):
        self.events: list[torch.cuda.Event] = []
        self.grads: list[tuple] = []  # (param, gradient storage) pairs produced on the side
        self.uses: dict[int, int] = {}  # forward uses per parameter since the last join
        self.finals: list = []  # callables the join queues after its wait
        self.active = False

    def reset(self) -> None:
        """Drop everything registered since the last join (a step abandoned before its join, e.g.
        a failed HIP-graph capture: none of its side-stream work ran)."""
        self.events.clear()
        self.grads.clear()
        self.uses.clear()
        self.finals.clear()
        self.active = False

    def use(self, param: torch.Tensor) -> None:
        self.uses[id(param)] = self.uses.get(id(param), 0) + 1

    def single_use(self, params) -> bool:
        """Every parameter entered the graph once (several uses get their gradients summed by
        autograd as they arrive, before any join)."""
        return all(self.uses.get(id(p), 0) == 1 for p in params)

    def add(self, event: torch.cuda.Event, grads=(), finalize=None) -> None:
        """finalize: queued on the joining stream after the wait (e.g. the fixed-order slab sums
        of gradients whose partials the side stream computed)."""
        self.events.append(event)
        self.grads.extend((p, g.data_ptr()) for p, g in grads)
        if finalize is not None:
            self.finals.append(finalize)

    def run_finals(self) -> None:
        """Queue the pending finalize callables on the current stream (after its waits)."""
        finals, self.finals = self.finals, []
        for f in finals:
            f()

    def join(self, stream: torch.cuda.Stream | None = None, claim=None) -> dict:
        """Wait for the side stream and queue the finalize callables.  claim: ids of parameters
        whose gradient sums the caller forms itself (optim.AdamW: tt_adamw_multi_ex); a finalize
        that exposes ``grad_parts()`` (slab partials) for parameters all in claim is not run, and
        its {id(param): (part pointer, stride, slabs, owner)} are returned instead."""
        for ev in self.events:
            (stream or torch.cuda.current_stream()).wait_event(ev)
        self.events.clear()
        deferred = {}
        if claim:
            keep = []
            for f in self.finals:
                if hasattr(f, "grad_parts") and all(id(p) in claim for p in f.params):
                    deferred.update(f.grad_parts())
                else:
                    keep.append(f)
            self.finals = keep
        with torch.cuda.stream(stream) if stream is not None else _nullctx():
            self.run_finals()
        self.uses.clear()
        grads, self.grads = self.grads, []
        for p, at in grads:  # autograd must have handed the side-stream buffer to .grad as is
            if p.grad is None or p.grad.data_ptr() != at:
                raise RuntimeError("twotower_amd: a side-stream gradient was copied or accumulated before "
                                   "its kernel ran (SideGrads needs .grad set to None before backward)")
        return deferred


def _nullctx():
    return contextlib.nullcontext()


def join_side_grads(params) -> None:
    """Make the current stream wait for every side-stream gradient of ``params``."""
    seen = set()
    for p in params:
        sg = getattr(p, "_tt_side_grads", None)
        if sg is not None and id(sg) not in seen:
            seen.add(id(sg))
            sg.join()


def lib() -> ctypes.CDLL:
    """Load the HIP library once.  Raises if it was not built (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"twotower_amd: {LIB_PATH} is missing; build it with `make -C twotower_amd/csrc` "
                    "(or __graft_entry__.build()).  There is no CPU fallback.")
            cdll = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            for name, (res, args) in _SIGNATURES.items():
                fn = getattr(cdll, name)
                fn.restype = res
                fn.argtypes = args
            _lib = cdll
    return _lib


def last_error() -> str:
    msg = lib().tt_last_error()
    return msg.decode() if msg else ""


def check(rc: int, name: str) -> None:
    if rc != 0:
        raise RuntimeError(f"twotower_amd: {name} failed (code {rc}): {last_error()}")


class OpTimer:
    """Optional HIP-event bracketing of every C-ABI call on the torch current stream (the stream
    the call launches on).  bench.py enables it over the timed region to get live per-op device
    times for the roofline figures.

    Stamp mode (``stamp_capture``): while a graph is being captured, every C-ABI call is bracketed
    by two tt_stamp kernels on its stream instead (HIP events cannot be recorded inside a captured
    graph on ROCm); each replay of that graph then rewrites the stamps, and ``stamp_summary``
    turns them into per-op device times of the replayed step."""

    def __init__(self):
        self.enabled = False
        self.events: dict[str, list] = {}
        self.stamping = False
        self.stamp_buf: torch.Tensor | None = None
        self.stamps: list[tuple[str, int]] = []

    def reset(self):
        self.events = {}

    @contextlib.contextmanager
    def stamp_capture(self, device, slots: int = 4096):
        """Around a graph capture: stamp every C-ABI call the capture records."""
        self.stamp_buf = torch.zeros(slots, dtype=torch.int64, device=device)
        self.stamps = []
        self.stamping = True
        try:
            yield
        finally:
            self.stamping = False

    def stamp_summary(self, device) -> dict[str, list[float]]:
        """Per op, its device time (ms) summed over its calls in the last replay of the stamped graph."""
        khz = lib().tt_wall_clock_khz(torch.device(device).index or 0)
        if khz <= 0:
            raise RuntimeError("tt_wall_clock_khz failed")
        t = self.stamp_buf.cpu().tolist()
        out: dict[str, list[float]] = {}
        for name, i in self.stamps:
            out.setdefault(name, []).append((t[i + 1] - t[i]) / khz)
        return out

    def run(self, name: str, fn):
        if torch.cuda.is_current_stream_capturing():
            if not self.stamping:
                return fn()
            i = 2 * len(self.stamps)
            if i + 2 > self.stamp_buf.numel():
                raise RuntimeError("OpTimer: stamp buffer full")
            s = torch.cuda.current_stream().cuda_stream
            check(lib().tt_stamp(self.stamp_buf.data_ptr() + 8 * i, s), "tt_stamp")
            rc = fn()
            check(lib().tt_stamp(self.stamp_buf.data_ptr() + 8 * (i + 1), s), "tt_stamp")
            self.stamps.append((name, i))
            return rc
        if not self.enabled:
            return fn()
        start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        start.record()
        rc = fn()
        end.record()
        self.events.setdefault(name, []).append((start, end))
        return rc

    def summary(self) -> dict[str, dict]:
        torch.cuda.synchronize()
        out = {}
        for name, evs in self.events.items():
            ms = [s.elapsed_time(e) for s, e in evs]
            out[name] = {"calls": len(ms), "mean_ms": sum(ms) / len(ms), "total_ms": sum(ms)}
        return out


TIMER = OpTimer()

# names of the C-ABI entry points called while a record_calls() block is open (tests and smoke()
# use it to show which kernels a path actually ran, e.g. the hand-written head vs the library one)
_CALLS: list[set] = []


@contextlib.contextmanager
def record_calls():
    seen: set = set()
    _CALLS.append(seen)
    try:
        yield seen
    finally:
        _CALLS.remove(seen)


def call(name: str, *args) -> None:
    fn = getattr(lib(), name)
    for seen in _CALLS:
        seen.add(name)
    if not (TIMER.enabled or TIMER.stamping):  # the common case: no per-op timing, no capture query
        check(fn(*args), name)
        return
    check(TIMER.run(name, lambda: fn(*args)), name)


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_of(t: torch.Tensor) -> int:
    """The raw handle of the current stream on t's device (without building a Stream object: this
    runs once per kernel launch on the eager paths)."""
    if _RAW_STREAM is not None and t.device.index is not None:
        return _RAW_STREAM(t.device.index)
    return torch.cuda.current_stream(t.device).cuda_stream


def require_gpu(*tensors: torch.Tensor) -> None:
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError("twotower_amd: the HIP kernels need GPU tensors (no CPU fallback); "
                               f"got a tensor on {t.device}")


def ids_dtype_code(ids: torch.Tensor) -> int:
    if ids.dtype == torch.int64:
        return TT_IDS_I64
    if ids.dtype == torch.int32:
        return TT_IDS_I32
    raise TypeError(f"token ids must be int32 or int64, got {ids.dtype}")


def compute_dtype_code(name) -> int:
    if isinstance(name, int):
        return name
    key = str(name).lower()
    if key not in COMPUTE_DTYPES:
        raise ValueError(f"unknown compute_dtype {name!r}; choose one of {sorted(COMPUTE_DTYPES)}")
    return COMPUTE_DTYPES[key]
