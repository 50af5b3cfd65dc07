#!/usr/bin/env python
"""Two-tower training-step benchmark on MI355X (driver contract: one JSON line from rank 0).

Workload (BASELINE.json configs[2], C3): V = 200k, E = H = d = 256, L = 64, B = 8192 queries per
GPU, each with one positive and one negative document (MS-MARCO-shaped synthetic ids resident
in HBM), tied mean-pool towers, in-batch sampled softmax over all 2B documents of the step
(candidates all-gathered across ranks when N > 1: configs[3], C4) on the bf16 MFMA scorer,
fp32 embedding gradient, AdamW over every parameter.  A step = forward (3 towers) + loss +
backward + gradient sync + optimizer step.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c4|c2|c5] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import twotower_amd as tt  # noqa: E402
from twotower_amd import _lib, ops as tt_ops  # noqa: E402

CONFIGS = {
    # name: V, E(=H), L, B (queries per GPU), scorer dtype, loss, negatives per query
    "c3": dict(V=200_000, d=256, L=64, B=8192, dtype="bf16", loss="in_batch", negatives=1,
               workload="C3: vocab 200k, d 256, seq 64, batch 8192, in-batch negatives (M = 2B), bf16 MFMA scorer, "
               "fp32 embedding grad"),
    # BASELINE.json configs[3] as SURVEY §8(a) a5 / §8(d) size it: (query, positive) pairs, every rank's
    # positives all-gathered as the candidates, M = N * B (65,536 at N = 8; 825 GFLOP per GPU)
    "c4": dict(V=200_000, d=256, L=64, B=8192, dtype="bf16", loss="in_batch", negatives=0,
               workload="C4 (pairs form): vocab 200k, d 256, seq 64, batch 8192 (query, positive) pairs per GPU, "
               "in-batch negatives over every rank's positives (M = N * B), bf16 MFMA scorer, fp32 embedding grad"),
    "c2": dict(V=50_000, d=128, L=32, B=4096, dtype="fp32", loss="in_batch", negatives=1,
               workload="C2: vocab 50k, d 128, seq 32, batch 4096, in-batch negatives (M = 2B), fp32"),
    # BASELINE.json configs[4] per GPU: presets/multi_pos_multi_neg.yml shape (1 positive + 4 negatives
    # per query = 6 sequences per query), vocab 1M; per-sample loss, so ranks exchange gradients only
    "c5": dict(V=1_000_000, d=256, L=64, B=8192, dtype="fp32", loss="multiple_negatives", negatives=4,
               workload="C5: vocab 1M, d 256, seq 64, batch 8192 queries x (1 positive + 4 negatives), "
               "multiple_negatives InfoNCE (cosine / 0.1, fp32), sorted scatter-add embedding grad fused with AdamW"),
}
# measured scorer gradient error at C3 (max over dq, dd; profiles/r02_scorer_error_table.jsonl)
SCORER_GRAD_ERROR = {
    ("bf16", True): {"vs_rounded_operands": 1.64e-5, "vs_fp32_operands": 3.11e-3},
    ("bf16", False): {"vs_rounded_operands": 1.64e-5, "vs_fp32_operands": 3.11e-3},
    ("bf16_split", False): {"vs_rounded_operands": 7.9e-8, "vs_fp32_operands": 3.11e-3},
    ("fp32", False): {"vs_fp32_operands": 9.7e-8},
}
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md chip table (spec)
MFMA_PEAK_TFLOPS = {"bf16": 2500.0, "fp32": 157.3}


def scorer_pmc(config: str) -> dict | None:
    """MFMA busy of the two scorer engines (SQ_VALU_MFMA_BUSY_CYCLES per SIMD-cycle) from the newest
    committed scorer PMC profile (profiles/<tag>_scorer_pmc.json, tools/pmc_scorer.sh +
    tools/pmc_report.py at the C3 scorer shape): the counter view of "MFMA utilisation", beside
    the algorithmic rate over every scorer kernel that `frac` reports."""
    import glob

    if config != "c3":
        return None
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_scorer_pmc.json")))
    if not files:
        return None
    d = json.load(open(files[-1]))
    out = {k: v.get("mfma_busy") for k, v in d.get("passes", {}).items()}
    out = {f"mfma_busy_{k}": v for k, v in out.items() if v is not None}
    if "engines_mfma_busy" in d:
        out["mfma_busy_engines"] = d["engines_mfma_busy"]
    # the clock each engine ran at while profiled: its known MFMA cycles per SIMD (C3 shape: B 8192,
    # M 16384, H 256; 32 cycles per 32x32x16 bf16 MFMA; forward 4BMH, stored-P backward 2BMH
    # executed) over busy fraction x duration -- the dense peak at that clock is 2.5 PF x f / 2.4 GHz
    B, M, H = 8192, 16384, 256
    for k, mult in (("fwd", 4), ("bwd", 2)):
        p = d.get("passes", {}).get(k, {})
        if p.get("mfma_busy") and p.get("engine_us"):
            cycles = mult * B * M * H / 32768 / 1024 * 32
            out[f"clock_ghz_{k}"] = round(cycles / (p["mfma_busy"] * p["engine_us"] * 1e-6) / 1e9, 3)
    out["source"] = os.path.relpath(files[-1], ROOT)
    return out


def pmc_traffic(abi: str, config: str) -> dict:
    """roofline.traffic: HBM bytes per launch of the dominant op from the newest committed PMC
    profile of this workload (profiles/<tag>_pmc_traffic.json, written by tools/profile_round.sh:
    FETCH_SIZE x2 + WRITE_SIZE over the op's kernels).  PMC counters cannot be read inside this
    process, so the figure comes from a separate rocprofv3 pass of this same command."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*{config}*_pmc_traffic.json")))
    for f in reversed(files):
        ops = json.load(open(f)).get("ops", {})
        if abi in ops and ops[abi].get("hbm_bytes_per_call"):
            return {"traffic": round(ops[abi]["hbm_bytes_per_call"]), "traffic_source": os.path.relpath(f, ROOT)}
    return {"traffic": None}


def gather_hbm_evidence(config: str, gather: dict | None, V: int, d: int) -> dict | None:
    """The gather's GB/s with what backs it: the C3 table (205 MB) fits the 256 MiB Infinity
    Cache, so its algorithmic rate is not an HBM figure; the C5 table (1.02 GB) does not, and the
    newest committed C5 profile (profiles/<tag>_c5_pmc_traffic.json: FETCH_SIZE x2 + WRITE_SIZE per
    launch, tools/profile_round.sh --config c5) gives counter-measured bytes over the kernel's
    time there, plus the C5 table update's counter-to-algorithmic traffic ratio."""
    import glob

    if gather is None:
        return None
    out = {"gbs": gather["achieved"], "table_bytes": V * d * 4, "mall_resident": V * d * 4 <= 256 * 2 ** 20,
           "basis": "algorithmic bytes / kernel time (HIP events), this run"}
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_c5_pmc_traffic.json")))
    if files:
        ops = json.load(open(files[-1])).get("ops", {})
        g, u = ops.get("tt_bag_mean_fwd"), ops.get("tt_bag_mean_bwd_adamw_planned")
        if g and g.get("device_us_per_step"):
            out["c5_counter_gbs"] = round(g["hbm_bytes_per_call"] / (g["device_us_per_step"] * 1e-6) / 1e9, 1)
            out["c5_counter_frac"] = round(out["c5_counter_gbs"] / HBM_PEAK_GBS, 4)
        if u and u.get("hbm_bytes_per_call"):
            c5 = CONFIGS["c5"]
            nseq = (2 + c5["negatives"]) * c5["B"]
            algo = nseq * c5["d"] * 4 + nseq * 4 + 24 * c5["V"] * c5["d"]
            out["c5_table_update_traffic_ratio"] = round(u["hbm_bytes_per_call"] / algo, 3)
        out["c5_source"] = os.path.relpath(files[-1], ROOT)
    return out


_MARK_BUF: dict = {}


def window_marker(dev) -> None:
    """One tt_stamp launch (a one-wave kernel, `stamp_kernel` in a trace) outside the timed region:
    the first two of a run bracket the timed steps, so tools/summarize_profile.py attributes only
    the kernels between them to the step (bench set-up, batch RNG and warmup left out)."""
    buf = _MARK_BUF.get(dev)
    if buf is None:
        buf = _MARK_BUF[dev] = torch.zeros(2, dtype=torch.int64, device=dev)
    tt_ops.call("tt_stamp", buf.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)


def sleep_cycles_per_ms(dev) -> float:
    """torch.cuda._sleep's spin rate on this device (cycles per ms), from one timed spin."""
    n = 2_000_000
    torch.cuda._sleep(n // 10)  # first launch
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    torch.cuda._sleep(n)
    en.record()
    torch.cuda.synchronize(dev)
    return n / max(st.elapsed_time(en), 1e-3)


def stamped_op_times(model, loss_fn, opt, batches, reps: int, dev) -> dict:
    """Per-op device times (ms per call) of the replayed step: a TrainStep captured with every
    C-ABI call bracketed by tt_stamp kernels (_lib.OpTimer.stamp_capture), replayed `reps` times,
    the stamps read after each replay.  Returns _lib.OpTimer.summary()'s format."""
    sstep = tt.TrainStep(model, loss_fn, opt, graph=True, eager_steps=1)
    sstep(*batches[0])  # eager: lazy set-up
    with _lib.TIMER.stamp_capture(dev):
        sstep(*batches[1])  # captured (stamped) and replayed once
    per: dict[str, list[float]] = {}
    for k in range(reps):
        sstep(*batches[k % len(batches)])
        torch.cuda.synchronize()
        for name, ts in _lib.TIMER.stamp_summary(dev).items():
            per.setdefault(name, []).extend(ts)
    return {n: {"calls": len(v), "mean_ms": sum(v) / len(v), "total_ms": sum(v)} for n, v in per.items()}


def normalise_ms(rows: int, d: int, dev, reps: int = 20) -> float:
    """Device time of the head's plain L2-normalise pass on (rows, d): tt_head_gemm with the
    normalise (epi 1) minus without it (epi 4), HIP events on the launch stream."""
    if d != tt_ops.HEAD_WIDTH:
        return 0.0
    g = torch.Generator(device=dev).manual_seed(0)
    h = torch.randn(rows, d, device=dev, generator=g)
    W = torch.randn(d, d, device=dev, generator=g) * 0.05
    b = torch.zeros(d, device=dev)
    planes = tt_ops._planes(W, False)
    norms = torch.empty(rows, device=dev)
    t = {}
    for epi in (1, 4, 1, 4):
        tt_ops._head_gemm(h, planes, epi, bias=b, norms=norms)
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(int(sleep_cycles_per_ms(dev) * 4.0))  # the host queues all reps first
        st.record()
        for _ in range(reps):
            tt_ops._head_gemm(h, planes, epi, bias=b, norms=norms)
        en.record()
        torch.cuda.synchronize()
        t[epi] = st.elapsed_time(en) / reps
    return max(0.0, t[1] - t[4])


def l2_backward_ms(rows: int, d: int, dev, reps: int = 20) -> float:
    """Device time of the head's plain F.normalize backward (tt_l2norm_bwd) on (rows, d), HIP
    events on the launch stream."""
    g = torch.Generator(device=dev).manual_seed(0)
    y = torch.nn.functional.normalize(torch.randn(rows, d, device=dev, generator=g), dim=1)
    dout = torch.randn(rows, d, device=dev, generator=g)
    norms = torch.ones(rows, device=dev)
    dx = torch.empty_like(y)
    args = lambda: (tt_ops.ptr(dout), tt_ops.ptr(y), tt_ops.ptr(norms), rows, d, tt_ops.ptr(dx),  # noqa: E731
                    torch.cuda.current_stream(dev).cuda_stream)
    t = 0.0
    for _ in range(2):
        tt_ops.call("tt_l2norm_bwd", *args())
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(int(sleep_cycles_per_ms(dev) * 4.0))  # the host queues all reps first
        st.record()
        for _ in range(reps):
            tt_ops.call("tt_l2norm_bwd", *args())
        en.record()
        torch.cuda.synchronize()
        t = st.elapsed_time(en) / reps
    return t


def scorer_entry(ops_t: dict, timing_steps: int, B: int, M: int, d: int, world: int, scorer_dtype: str,
                 bwd_form: str, normalise=lambda: 0.0, l2_backward=lambda: 0.0) -> dict | None:
    """The in-batch scorer's roofline entry (B queries x M candidates, width d) from per-op
    device times: both passes, the operand prep's cost beyond a plain normalise and the fused
    backward's cost beyond a plain L2 backward."""
    pk = MFMA_PEAK_TFLOPS["fp32" if scorer_dtype == "fp32" else "bf16"]
    mult = 2 if scorer_dtype == "bf16_split" else 1  # hi/lo P doubles the second product
    # single process, bf16 or fp32: the backward reads the forward's stored probabilities (no S recompute)
    stored_p = world == 1 and bwd_form == "stored" and (
        (scorer_dtype == "bf16" and B * M <= 2 ** 31) or (scorer_dtype == "fp32" and B * M <= 2 ** 30))
    fwd_key = "tt_inbatch_fwd_prepped" if "tt_inbatch_fwd_prepped" in ops_t else "tt_inbatch_fwd"
    bwd_key = "tt_inbatch_bwd_l2" if "tt_inbatch_bwd_l2" in ops_t else "tt_inbatch_bwd"
    if fwd_key not in ops_t or bwd_key not in ops_t:
        return None
    # one entry for both passes: the forward also forms P.D (dQ's product), so a per-pass split
    # of the 2BMH + 4BMH algorithmic flops would credit the backward with work the forward did
    fwd_ms, bwd_ms = ops_t[fwd_key]["mean_ms"], ops_t[bwd_key]["mean_ms"]
    l2_ms = None
    if bwd_key == "tt_inbatch_bwd_l2":
        # the backward combine also runs the tower head's F.normalize backward: the scorer is
        # charged what that pass costs beyond a plain tt_l2norm_bwd over the same rows
        l2_ms = l2_backward()
        bwd_ms = max(0.0, bwd_ms - l2_ms)
    prep_ms = None
    if fwd_key == "tt_inbatch_fwd_prepped" and "tt_inbatch_l2_prep" in ops_t:
        # the operand prep runs inside the head's normalise pass (tt_inbatch_l2_prep): charge
        # the scorer what that pass costs beyond the plain normalise, measured on the same rows
        prep_ms = max(0.0, ops_t["tt_inbatch_l2_prep"]["mean_ms"] - normalise())
    ms = fwd_ms + bwd_ms + (prep_ms or 0.0)
    algo = 6.0 * B * M * d
    executed = ((2.0 + 2.0 * mult) + (2.0 if stored_p else 2.0 + 2.0 * mult)) * B * M * d
    achieved = algo / (ms * 1e-3) / 1e12
    # fp32 stored-P passes at H 64 / 128 / 256 run the split-bf16 engines: six bf16 MFMA products per
    # fp32 product, so the peak their instruction mix can reach is the bf16 peak / 6 (a
    # fraction against the 157 TF fp32 MFMA rate above 1 said nothing about the engines)
    split_engines = scorer_dtype == "fp32" and stored_p and d in (64, 128, 256)
    extra = {}
    if split_engines:
        extra = {"peak_basis": "split-bf16 engines: 2.5 PF bf16 / 6 products per fp32 product",
                 "frac_vs_fp32_mfma_157tf": round(achieved / MFMA_PEAK_TFLOPS["fp32"], 4)}
        pk = MFMA_PEAK_TFLOPS["bf16"] / 6.0
    form = (f"{scorer_dtype}, backward from stored {scorer_dtype} probabilities" if stored_p else
            {"bf16": "bf16, recompute backward", "bf16_split": "bf16 with hi/lo-split probabilities",
             "fp32": "fp32 MFMA, recompute backward"}[scorer_dtype])
    return {
        "op": "in-batch scorer, forward + backward (prep, MFMA engines, combines)",
        "abi": fwd_key + "+" + bwd_key, "bound": "mfma", "mean_ms": round(ms, 4), "B": B, "M": M,
        "pass_ms": {"forward": round(fwd_ms, 4), "backward": round(bwd_ms, 4),
                    **({"operand_prep_in_head_normalise": round(prep_ms, 4)} if prep_ms is not None else {}),
                    **({"plain_l2_backward_subtracted": round(l2_ms, 4)} if l2_ms is not None else {})},
        "calls_per_step": ops_t[fwd_key]["calls"] / timing_steps, "achieved": round(achieved, 2),
        "peak": pk, "unit": "TFLOP/s", "frac": round(achieved / pk, 4), "algorithmic": algo,
        "executed": executed, "executed_rate": round(executed / (ms * 1e-3) / 1e12, 2),
        "per_launch": "6*B*M*H algorithmic flops (2BMH S + 4BMH dQ, dD) over both passes",
        "form": form,
        # measured max-abs-normalised gradient error at C3 (tools/scorer_error_table.py --big,
        # profiles/r02_scorer_error_table.jsonl): against float64 on the same bf16-rounded
        # operands, and against float64 on the fp32 operands (what the reference computes)
        "grad_error": SCORER_GRAD_ERROR.get((scorer_dtype, stored_p)),
        **extra,
    }


def op_report(ops_t: dict, timing_steps: int, config: str, world: int, scorer_dtype: str, nnz: float,
              tower_params: int, bwd_form: str, normalise=lambda: 0.0, l2_backward=lambda: 0.0):
    """Per-op rooflines from the per-op device times (HIP events on each C-ABI call's launch
    stream, ops_t = _lib.TIMER.summary()) and the dominant main-stream op's roofline."""
    cfg = CONFIGS[config]
    V, d, L, B, K = cfg["V"], cfg["d"], cfg["L"], cfg["B"], cfg["negatives"]
    nseq = (2 + K) * B
    M = (1 + K) * B * world if cfg["loss"] == "in_batch" else K + 1
    kernels = []

    def add(name, key, algo, unit, peak, bound, per_launch_note, side_stream=False, executed=None):
        if key not in ops_t:
            return
        ms = ops_t[key]["mean_ms"]
        achieved = algo / (ms * 1e-3) / (1e9 if unit == "GB/s" else 1e12)
        k = {"op": name, "abi": key, "bound": bound, "mean_ms": round(ms, 4),
             "calls_per_step": ops_t[key]["calls"] / timing_steps, "achieved": round(achieved, 2),
             "peak": peak, "unit": unit, "frac": round(achieved / peak, 4), "algorithmic": algo,
             "per_launch": per_launch_note}
        if executed is not None:  # work the kernels do beyond the algorithmic count (e.g. P.D in the forward)
            k["executed"] = executed
            k["executed_rate"] = round(executed / (ms * 1e-3) / 1e12, 2)
        if side_stream:  # its event span covers the overlap with the forward, not its kernels alone
            k["stream"] = "side (overlapped)"
        kernels.append(k)

    id_bytes = 4  # int32 ids on device
    add("embedding bag forward (gather + masked mean)", "tt_bag_mean_fwd",
        nseq * L * id_bytes + nnz * d * 4 + nseq * d * 4 + nseq * 4, "GB/s", HBM_PEAK_GBS, "hbm",
        "ids N*L*4 + gathered rows nnz*E*4 + pooled N*E*4 + denom N*4 bytes")
    # the same gather whose launch also splits the head's weights into bf16 planes (the encoders'
    # default for the hand-written head): W1, W2 read twice (direct, transposed), 12 B of planes each
    add("embedding bag forward (gather + masked mean) + head weight planes", "tt_bag_mean_fwd_split",
        nseq * L * id_bytes + nnz * d * 4 + nseq * d * 4 + nseq * 4 + 2 * d * d * (8 + 12), "GB/s", HBM_PEAK_GBS,
        "hbm", "ids N*L*4 + gathered rows nnz*E*4 + pooled N*E*4 + denom N*4 + W1, W2 (E = H) 2 x 4 B read "
        "and 2 x 6 B of bf16 planes written per weight element")
    add("embedding bag backward fused with table AdamW (apply half: scale rows + per-row reduce + AdamW)",
        "tt_bag_mean_bwd_adamw_planned", nseq * d * 4 + nseq * 4 + 24 * V * d, "GB/s", HBM_PEAK_GBS, "hbm",
        "d_pooled N*E*4 + denom N*4 + AdamW p,m,v read+write 24*V*E bytes")
    add("embedding bag backward sort plan (ids -> sorted (row, seq) + segments; side stream, overlaps the towers)",
        "tt_bag_plan", nseq * L * 4 + nnz * 8 + V * 8, "GB/s", HBM_PEAK_GBS, "hbm",
        "ids N*L*4 + sorted (row, seq) pairs nnz*8 + segment bounds V*8 bytes (latency-bound radix sort)",
        side_stream=True)
    add("embedding bag backward (dense grad, apply half)", "tt_bag_mean_bwd_planned",
        nseq * d * 4 + nseq * 4 + V * d * 4, "GB/s", HBM_PEAK_GBS, "hbm", "d_pooled + denom + V*E*4 grad write")
    sc = scorer_entry(ops_t, timing_steps, B, M, d, world, scorer_dtype, bwd_form, normalise, l2_backward)
    if sc is not None:
        kernels.append(sc)
        if scorer_dtype == "bf16" and world == 1:
            pmc = scorer_pmc(config)
            if pmc:
                kernels[-1]["pmc"] = pmc
    add("multiple-negatives loss forward (cosines + CE)", "tt_multi_neg_fwd", (2 + K) * B * d * 4 + B * 4, "GB/s",
        HBM_PEAK_GBS, "hbm", "q, p, negatives read (2 + K)*B*H*4 + loss rows B*4 bytes")
    add("multiple-negatives loss backward", "tt_multi_neg_bwd", 2 * (2 + K) * B * d * 4, "GB/s", HBM_PEAK_GBS, "hbm",
        "q, p, negatives read + their gradients written 2*(2 + K)*B*H*4 bytes")
    add("dense AdamW (tower FF, multi-tensor)", "tt_adamw_multi", 28 * tower_params, "GB/s", HBM_PEAK_GBS, "hbm",
        "28 bytes per parameter")
    # the step's fused tail: the head weight gradients' slab sums (2 x 32 slabs of 256 x 257
    # partials read, the gradients written) + the dense AdamW + the next step's scalars
    add("step tail: head weight-gradient slab sums + dense AdamW + next scalars", "tt_adamw_multi_ex",
        28 * tower_params + 2 * 32 * 256 * 257 * 4 + 2 * 256 * 257 * 4, "GB/s", HBM_PEAK_GBS, "hbm",
        "28 bytes per parameter + 2*32*256*257*4 partial bytes read + 2*256*257*4 gradient bytes written")
    # the tower head (encoders.py:38-42,77) on split-bf16 MFMA: six bf16 products per fp32 product,
    # so its MFMA peak is the dense bf16 peak / 6; algorithmic flops = the fp32 GEMM's 2 * rows * K * N
    split_peak = MFMA_PEAK_TFLOPS["bf16"] / 6.0
    add("tower head activation GEMMs (Linear-ReLU-Linear fwd, dh / dx bwd; split-bf16 MFMA, fused epilogues)",
        "tt_head_gemm", 2.0 * nseq * d * d, "TFLOP/s", split_peak, "mfma",
        "2*rows*E*H fp32-GEMM flops per launch (4 launches per step); peak = 2.5 PF bf16 / 6 (six bf16 products "
        "per fp32 product)")
    add("tower head weight + bias gradients (dW1, dW2 as one launch; side stream beside the table update)",
        "tt_head_wgrad2", 4.0 * nseq * d * d, "TFLOP/s", split_peak, "mfma",
        "2 x 2*rows*E*H fp32-GEMM flops (dW1 and dW2 = G^T X); peak = 2.5 PF bf16 / 6", side_stream=True)
    add("tower head weight + bias gradient (one Linear)", "tt_head_wgrad_ex", 2.0 * nseq * d * d, "TFLOP/s",
        split_peak, "mfma", "2*rows*E*H fp32-GEMM flops (dW = G^T X); peak = 2.5 PF bf16 / 6", side_stream=True)
    main_stream = [k for k in kernels if "stream" not in k]
    dominant = max(main_stream, key=lambda k: k["mean_ms"] * k["calls_per_step"]) if main_stream else None
    roofline = None
    if dominant:
        roofline = {"bound": dominant["bound"], "achieved": dominant["achieved"], "peak": dominant["peak"],
                    "unit": dominant["unit"], "frac": dominant["frac"], "traffic": None, "op": dominant["op"]}
        roofline.update(pmc_traffic(dominant["abi"], config))
    return kernels, roofline


class PlainLoop:
    """The reference's hot loop body unchanged (twotower/train.py:103-154) around this package's
    registry entries: eager ``model(q, p, n)`` (:120-122), ``loss_fn(q, p, n)`` (:133),
    ``optimizer.zero_grad(); loss.backward(); optimizer.step()`` (:137-139) with the reference's
    own ``torch.optim.AdamW(model.parameters(), lr)`` (:358-359: a dense V x E table gradient and
    torch's foreach AdamW over it), and the per-batch monitors: two cosine-similarity means and the
    loss, three ``.item()`` host syncs (:144-154).  What a user gets by swapping the registries
    and nothing else.  table_update "backward": the same loop with the config opt-in
    ``hip: {table_update: backward}`` (optim.fuse_table_update: the table's fused scatter + AdamW at
    the end of each backward, torch's AdamW for the towers)."""

    def __init__(self, model, loss_fn, lr: float = 1e-3, table_update: str = "optimizer"):
        self.model, self.loss_fn = model, loss_fn
        self.optimizer = torch.optim.AdamW(model.parameters(), lr=lr)
        if table_update in ("backward", "backward_all"):
            tt.optim.fuse_table_update(self.optimizer, model)
        if table_update == "backward_all":  # hip: {table_update: backward, dense_update: backward}
            tt.optim.fuse_dense_update(self.optimizer, model)

    def __call__(self, q, p, n=None):
        ins = (q, p) if n is None else (q, p, n)
        outs = self.model(*ins)
        loss = self.loss_fn(*outs)
        self.optimizer.zero_grad()
        loss.backward()
        self.optimizer.step()
        with torch.no_grad():
            pos = torch.nn.functional.cosine_similarity(outs[0], outs[1]).mean().item()
            neg = (torch.nn.functional.cosine_similarity(outs[0][:, None, :], outs[2].view(
                outs[0].shape[0], -1, outs[0].shape[1]), dim=-1).mean().item() if n is not None else 0.0)
            _ = pos - neg
        return torch.tensor(loss.item())

    eager = __call__


def time_steps(step, batches, steps: int, warmup: int) -> float:
    """ms per step of `step` over `steps` calls after `warmup`, synchronised at both ends."""
    for k in range(warmup):
        step(*batches[k % len(batches)])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        step(*batches[k % len(batches)])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def build_model(cfg, dev):
    torch.manual_seed(1234)  # identical initial weights on every rank
    emb = tt.embeddings.build("lookup", vocab_size=cfg["V"], embedding_dim=cfg["d"])
    model = tt.build_two_tower("mean", emb, hidden_dim=cfg["d"], tied_weights=True).to(dev)
    return emb, model


def bxb_scorer(cfg, scorer_dtype: str, dev, reps: int, steps: int, helpers: bool) -> dict | None:
    """The north_star's B x B scorer (B = 8192 queries against their own 8192 positives, d 256):
    the (query, positive) pairs form of the same fused step (TwoTower(q, d) + the in-batch loss
    over the positives, M = B), graph-replayed.  Per-op times from a stamped replay as for the
    main line; the step's own time and pairs/s beside it (the C4 pairs form at one GPU)."""
    if cfg["loss"] != "in_batch":
        return None
    B, L, V, d = cfg["B"], cfg["L"], cfg["V"], cfg["d"]
    emb, model = build_model(cfg, dev)
    opt = tt.optim.AdamW(model.parameters(), lr=1e-3, fused_tables=True, tables=[emb], capturable=True)
    loss_fn = tt.losses.build("in_batch", temperature=0.1, compute_dtype=scorer_dtype)
    batches = [tt.data.synthetic_triplets(B, L, V, seed=700 + k, device=dev)[:2] for k in range(4)]
    step = tt.TrainStep(model, loss_fn, opt, graph=True)
    ms = time_steps(step, batches, steps, 5)
    ops_t = stamped_op_times(model, loss_fn, opt, batches, reps, dev)
    e = scorer_entry(ops_t, reps, B, B, d, 1, scorer_dtype, tt_ops.get_inbatch_backward(),
                     *((lambda: normalise_ms(2 * B, d, dev), lambda: l2_backward_ms(2 * B, d, dev)) if helpers else ()))
    if e is None:
        return None
    e["op"] = "in-batch scorer, B x B (M = B: query, positive pairs), forward + backward"
    e["step_ms"] = round(ms, 4)
    e["step_pairs_per_s"] = round(B / (ms * 1e-3), 1)
    e["workload"] = (f"pairs form of configs[2]: B {B} queries x their {B} positives, d {d}, L {L}, V {V}, "
                     f"{scorer_dtype} scorer; TwoTower(q, d) + in_batch, fused table AdamW, HIP graph")
    del step, opt, model, emb
    return e


def c4_pairs_entry(cfg, scorer_dtype: str, dev, world: int, rank: int, steps: int, warmup: int, table_sync: str,
                   use_graph: bool) -> dict:
    """BASELINE.json configs[3] as it is stated (N ranks): (query, positive) pairs, every rank's positives
    all-gathered as the candidates, M = N * B (65,536 global negatives at N = 8), timed like the main
    line (barrier + synchronize around the steps, max over ranks).  The main line at N ranks keeps the
    triplet form of configs[2] (M = N * 2B), so both C4 forms are reported."""
    B, L, V, d = cfg["B"], cfg["L"], cfg["V"], cfg["d"]
    emb, model = build_model(cfg, dev)
    opt = tt.optim.AdamW(model.parameters(), lr=1e-3, fused_tables=True, tables=[emb], capturable=True,
                         table_sync=table_sync)
    loss_fn = tt.losses.build("in_batch", temperature=0.1, compute_dtype=scorer_dtype, cross_device_negatives=True)
    step = tt.TrainStep(model, loss_fn, opt, graph=use_graph)
    batches = [tt.data.synthetic_triplets(B, L, V, seed=rank * 1000 + 500 + k, device=dev)[:2] for k in range(4)]
    for k in range(warmup):
        step(*batches[k % len(batches)])
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        step(*batches[k % len(batches)])
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms = float(t.item()) / steps * 1e3
    step.release()  # a captured all-to-all holds RCCL resources until its graph goes
    del step, opt, model, emb
    return {"value": round(B * world / (ms * 1e-3), 1), "unit": "pairs/s", "ms_per_step": round(ms, 4),
            "steps": steps, "warmup": warmup, "M": B * world,
            "workload": f"C4 pairs form (configs[3]): {world} x {B} (query, positive) pairs, candidates = every "
                        f"rank's positives (M = {B * world}), d {d}, L {L}, V {V}, {scorer_dtype} scorer, "
                        f"table_sync {table_sync}, {'HIP graph' if use_graph else 'eager'}"}


def plain_loop_entry(cfg, loss_fn, batches, dev, steps: int, trainstep_ms: float) -> dict:
    """PlainLoop timed on the bench's batches (fresh model, torch.optim.AdamW), as is and with the
    config opt-in hip: {table_update: backward}."""
    out = {}
    for mode in ("optimizer", "backward", "backward_all"):
        _, model = build_model(cfg, dev)
        loop = PlainLoop(model, loss_fn, table_update=mode)
        ms = time_steps(loop, batches, steps, 3)
        del loop, model
        out[mode] = {"ms_per_step": round(ms, 4), "pairs_per_s": round(cfg["B"] / (ms * 1e-3), 1),
                     "slowdown_vs_trainstep": round(ms / trainstep_ms, 3)}
    e = dict(out["optimizer"])
    e.update({"steps": steps, "trainstep_ms_per_step": round(trainstep_ms, 4),
              "loop": "twotower/train.py:103-154 body unchanged: eager model(q,p,n), loss_fn, zero_grad/backward/"
                      "step with torch.optim.AdamW(model.parameters(), lr=1e-3) (dense V x E table gradient), "
                      "cosine monitors + 3 .item() syncs per step",
              "table_update_backward": dict(out["backward"], config="hip: {table_update: backward} (the same loop; the "
                                            "table's fused scatter + AdamW at the end of loss.backward(), torch's "
                                            "AdamW for the towers)"),
              "table_and_dense_update_backward": dict(
                  out["backward_all"], config="hip: {table_update: backward, dense_update: backward} (the same loop; "
                  "the towers' AdamW too as one multi-tensor launch at the end of loss.backward(), optimizer.step() "
                  "then has nothing left)")})
    return e


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)  # >= 50 timed steps after 10 warm-up
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--scorer-dtype", default=None, help="override: fp32 | bf16 | bf16_split")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                    help="replay the step as one HIP graph (auto: on for a single GPU)")
    ap.add_argument("--force-dist", action="store_true",
                    help="rehearsal: one rank runs every data-parallel exchange of the N-rank step (RCCL at world "
                         "size 1, TT_DIST_FORCE=1), e.g. to check the N-rank step under HIP-graph capture on one GPU")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL over xGMI) for real runs; gloo only to rehearse N ranks on one GPU")
    ap.add_argument("--table-sync", default="best", choices=["best", "auto", "gather", "shard", "owner", "column"],
                    help="N ranks: table update from gathered ids + row grads on every rank (gather), row-sharded "
                         "AdamW after a gradient reduce-scatter (shard), each rank's own rows from the gathered "
                         "factored gradient (owner), or each rank's own columns of every row (column); auto (the "
                         "library default) picks gather up to 4 ranks, shard beyond; best (this bench's default) "
                         "takes column wherever the width splits into the column kernels' slabs, else auto")
    ap.add_argument("--timing-steps", type=int, default=10, help="eager steps timed per op after the timed region")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-batch", type=int, default=8192,
                    help="queries per CPU step (the full per-GPU batch: the dense AdamW over the table is a "
                         "fixed per-step cost, so a smaller batch would understate the CPU rate)")
    ap.add_argument("--no-helpers", action="store_true",
                    help="skip the scorer-attribution helper timings (normalise / plain L2 backward on the same rows): "
                         "tools/profile_round.sh sets it so every kernel in the trace belongs to a step")
    ap.add_argument("--zipf", type=float, default=None,
                    help="token ids ~ Zipf(s) over the vocabulary (text-like hot rows); default uniform")
    ap.add_argument("--table-update", default="optimizer", choices=["optimizer", "backward", "backward_all"],
                    help="--loop plain: the config opt-in hip: {table_update: backward} (fused table update in "
                         "backward); backward_all adds hip: {dense_update: backward} (the towers' AdamW too)")
    ap.add_argument("--loop", default="trainstep", choices=["trainstep", "plain"],
                    help="plain: time the reference's loop body unchanged (bench.PlainLoop: eager, torch.optim.AdamW, "
                         "three .item() syncs) instead of TrainStep")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the B x B scorer entry and the plain-loop entry measured after the timed region")
    return ap.parse_args()


def child_world_env(dev) -> dict:
    """Environment for a child process of every rank that forms its own process group of the same
    ranks: a free port chosen by rank 0 and broadcast, and its own store (under torch.distributed.run
    TORCHELASTIC_USE_AGENT_STORE=True would make every child a client of the agent's store on the
    job's port, where nothing serves the new one)."""
    import socket

    port = 0
    if dist.get_rank() == 0:
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
    t = torch.tensor([port], dtype=torch.int64, device=dev)
    if dist.get_world_size() > 1:
        dist.broadcast(t, 0)
    env = dict(os.environ)
    env["MASTER_PORT"] = str(int(t.item()))
    env["TORCHELASTIC_USE_AGENT_STORE"] = "False"
    return env


def dp_capture_canary(cfg, scorer_dtype: str, table_sync: str, dev) -> str:
    """Run tools/dp_capture_canary.py as a child of this rank (its own RCCL world of the same
    ranks, every rank's child together); "ok" if this rank's child captured and replayed the small
    N-rank step."""
    env = child_world_env(dev)
    cmd = [sys.executable, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools", "dp_capture_canary.py"),
           "--d", str(cfg["d"]), "--loss", cfg["loss"], "--negatives", str(cfg["negatives"]), "--dtype", scorer_dtype,
           "--table-sync", table_sync]
    try:
        r = subprocess.run(cmd, env=env, timeout=240, capture_output=True, text=True)
    except subprocess.TimeoutExpired:
        return "timeout"
    if r.returncode == 0 and "canary ok" in r.stdout:
        return "ok"
    return f"failed (rc {r.returncode})"


def setup_dist(backend: str, force: bool = False):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend == "gloo":  # rehearsal of the DP path on one GPU (ranks share it); RCCL is the real path
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if force and world == 1:  # one-rank rehearsal of every collective (distributed.is_active)
        os.environ["TT_DIST_FORCE"] = "1"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29561")
        kw = {"device_id": torch.device("cuda", local)} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=0, world_size=1, **kw)
        return world, rank
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank


def main():
    args = parse()
    world, rank = setup_dist(args.dist_backend, args.force_dist)
    dp = world > 1 or args.force_dist
    cfg = CONFIGS[args.config]
    V, d, L, B = cfg["V"], cfg["d"], cfg["L"], cfg["B"]
    scorer_dtype = args.scorer_dtype or cfg["dtype"]
    dev = torch.device("cuda", torch.cuda.current_device())
    if args.table_sync == "best":  # the scaling choice, opt-in in the library
        args.table_sync = "column" if dp and tt.distributed.column_ok(d, max(world, 1)) else "auto"

    emb, model = build_model(cfg, dev)
    K = cfg["negatives"]
    if cfg["loss"] == "in_batch":
        loss_fn = tt.losses.build("in_batch", temperature=0.1, compute_dtype=scorer_dtype,
                                  cross_device_negatives=dp)
    else:  # multiple_negatives over (q, p, n viewed as (B, K, H)); per-sample, no cross-rank exchange
        mn = tt.losses.build("multiple_negatives", temperature=0.1)

        def loss_fn(q, p, n):
            return mn(q, p, n.view(q.shape[0], K, q.shape[1]))
    # the step is one HIP graph; N ranks (nccl) only after every rank's child process has captured
    # and replayed a small N-rank step through the same paths (tools/dp_capture_canary.py), so a
    # capture that fails or crashes on the box's ROCm/RCCL stack leaves this run eager
    canary = None
    plain = args.loop == "plain"
    use_graph = not plain and (args.graph == "on" or (args.graph == "auto" and not dp))
    if dp and not plain and args.graph == "auto" and args.dist_backend == "nccl":
        canary = dp_capture_canary(cfg, scorer_dtype, args.table_sync, dev)
        agree = torch.tensor([1 if canary == "ok" else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(agree, op=dist.ReduceOp.MIN)
        use_graph = bool(agree.item())
    if plain:
        if dp:
            raise SystemExit("--loop plain runs one GPU (the reference loop has no data parallelism)")
        opt, step = None, PlainLoop(model, loss_fn, table_update=args.table_update)
    else:
        # one rank: scatter fused with the table AdamW; N ranks: table rows sharded over the ranks
        # (reduce-scatter, AdamW on own rows, all-gather), tower grads all-reduced
        opt = tt.optim.AdamW(model.parameters(), lr=1e-3, fused_tables=True, tables=[emb], capturable=True,
                             table_sync=args.table_sync)
        step = tt.TrainStep(model, loss_fn, opt, graph=use_graph)

    batches = [tt.data.synthetic_triplets(B, L, V, seed=rank * 1000 + k, device=dev, zipf_s=args.zipf,
                                          negatives=max(K, 1))[:(2 if K == 0 else 3)]
               for k in range(4)]
    nnz = sum(int((t > 0).sum()) for b in batches for t in b) / len(batches)  # tokens per step

    for k in range(args.warmup):
        step(*batches[k % len(batches)])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    window_marker(dev)  # a profiler's trace of this run is cut to the timed steps at these markers
    torch.cuda.synchronize()

    t0 = time.perf_counter()
    loss = None
    for k in range(args.steps):
        loss = step(*batches[k % len(batches)])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    window_marker(dev)
    torch.cuda.synchronize()

    # Per-op device times for the rooflines, after the timed region (--timing-steps 0: none, e.g.
    # under rocprofv3, whose trace then holds the timed steps alone).
    if args.timing_steps <= 0:
        ops_t, timing_source = {}, None
    elif use_graph and world == 1:
        # From the replayed graph itself: a second capture of the same step with every C-ABI call
        # bracketed by tt_stamp kernels on its launch stream (HIP events cannot be recorded inside
        # a captured graph on ROCm); each replay rewrites the stamps.  Same kernels, same streams,
        # same overlap as the timed replays, plus two one-wave stamp kernels per op.
        ops_t, timing_source = stamped_op_times(model, loss_fn, opt, batches, args.timing_steps, dev), "graph_stamps"
    else:
        # Eager pass of the same step, HIP events around every C-ABI call on its launch stream.  Each
        # eager step is queued behind a spin kernel (torch.cuda._sleep) long enough for the host to
        # enqueue the whole step first: the GPU then runs the step back to back and an op's events
        # span its kernels, not the host's launch gaps (an eager step costs more host time than GPU).
        prime = sleep_cycles_per_ms(dev) * 8.0
        _lib.TIMER.reset()
        _lib.TIMER.enabled = True
        for k in range(args.timing_steps):
            torch.cuda._sleep(int(prime))
            step.eager(*batches[k % len(batches)])
        torch.cuda.synchronize()
        _lib.TIMER.enabled = False
        ops_t, timing_source = _lib.TIMER.summary(), "eager_events_primed"
    timing_steps = args.timing_steps

    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    # N ranks: configs[3] as stated (pairs form, M = N B) beside the main line's triplet form
    c4p = None
    if world > 1 and args.config == "c3" and not plain and not args.no_extras:
        c4p = c4_pairs_entry(cfg, scorer_dtype, dev, world, rank, max(args.steps, 1), max(args.warmup, 1),
                             args.table_sync, use_graph)
    ms_per_step = elapsed / args.steps * 1e3
    value = B * world * args.steps / elapsed

    if hasattr(step, "release"):  # the captured graphs go before the process group (RCCL resources)
        step.release()
    if rank != 0:
        if dist.is_initialized():
            dist.destroy_process_group()
        return

    M = (1 + K) * B * world if cfg["loss"] == "in_batch" else K + 1  # candidates per query
    kernels, roofline = op_report(ops_t, timing_steps, args.config, world, scorer_dtype, nnz,
                                  sum(p.numel() for n_, p in model.named_parameters() if "embedding" not in n_),
                                  tt_ops.get_inbatch_backward(),
                                  *(() if args.no_helpers else (lambda: normalise_ms((2 + K) * B, d, dev),
                                                                lambda: l2_backward_ms((2 + K) * B, d, dev))))
    gather = next((k for k in kernels if k["abi"] in ("tt_bag_mean_fwd", "tt_bag_mean_fwd_split")), None)

    # After the timed region, one GPU: the north_star's B x B scorer (the pairs form of the same
    # step, M = B) and the reference's loop body unchanged around these registries (PlainLoop)
    bxb, plain_entry = None, None
    if world == 1 and not dp and not plain and not args.no_extras:
        bxb = bxb_scorer(cfg, scorer_dtype, dev, max(args.timing_steps, 1), args.steps, not args.no_helpers)
        plain_entry = plain_loop_entry(cfg, loss_fn, batches, dev, 10, ms_per_step)

    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        from oracle.cpu_step import host_cores, time_cpu_step  # CPU baseline only: the GPU path never uses it

        cb = args.cpu_batch
        cpu_batches = [tuple(t[:cb].to("cpu", torch.int64) for t in b) for b in batches[:2]]  # (q, p[, n])
        if K > 1:
            cpu_batches = [tuple(t.to("cpu", torch.int64) for t in (b[0][:cb], b[1][:cb], b[2][:cb * K]))
                           for b in batches[:2]]
        hc = host_cores()
        # all physical host cores.  The box's CPU share may be smaller than the cores
        # it shows, so a short sweep over thread counts up to every physical core picks the count
        # the full-length measurement then runs at (the sweep is reported beside it).
        counts = sorted({c for c in (16, 32, 64, 128, hc["physical_cores"]) if c <= hc["physical_cores"]}
                        or {hc["physical_cores"]})
        sweep = {n: time_cpu_step(V, d, d, cpu_batches, loss=cfg["loss"], threads=n, min_seconds=1.0,
                                  max_steps=2)["pairs_per_s"] for n in counts}
        best = max(sweep, key=sweep.get)
        r = time_cpu_step(V, d, d, cpu_batches, loss=cfg["loss"], threads=best, min_seconds=args.cpu_seconds)
        # C1 (BASELINE.json configs[0]: configs/char_tower.yml, char vocab 34, E 64, H 128, triplet,
        # batch 64, L 64): the reference's own CPU configuration, a few seconds; a batch of 64 is
        # too small for many threads, so it gets its own short sweep
        c1_batches = [tuple(t.long() for t in tt.data.synthetic_triplets(64, 64, 34, seed=k, device="cpu"))
                      for k in range(2)]
        c1_counts = sorted({c for c in (1, 4, 16, best) if c <= hc["physical_cores"]})
        c1_sweep = {n: time_cpu_step(34, 64, 128, c1_batches, loss="triplet", threads=n, min_seconds=0.5,
                                     max_steps=500)["pairs_per_s"] for n in c1_counts}
        c1_best = max(c1_sweep, key=c1_sweep.get)
        r1 = time_cpu_step(34, 64, 128, c1_batches, loss="triplet", threads=c1_best, min_seconds=3.0, max_steps=5000)
        cpu = {"value": round(r["pairs_per_s"], 1), "unit": "pairs/s", "cores": r["threads"], "kind": "port",
               "physical_cores": hc["physical_cores"], "logical_cpus": hc["logical_cpus"],
               "threads_sweep": {str(n): round(v, 1) for n, v in sweep.items()},
               "sample": f"torch-CPU restatement of the reference step (oracle/cpu_step.py: train.py's step "
                         f"body incl. its per-batch monitors, within 1-8 % of the reference's own train_epoch "
                         f"on the same cores, profiles/r02_cpu_baseline_validation.json), same V/d/L, batch "
                         f"{min(cb, B)}" + (f" instead of {B}" if cb < B else "") + f", {cfg['loss']} loss fp32, "
                         f"{r['steps']} steps in {r['seconds']:.1f}s on {r['threads']} threads (the fastest of a "
                         f"{'/'.join(map(str, counts))}-thread sweep over the {hc['physical_cores']} physical cores)",
               "c1": {"value": round(r1["pairs_per_s"], 1), "unit": "pairs/s", "cores": r1["threads"],
                      "threads_sweep": {str(n): round(v, 1) for n, v in c1_sweep.items()},
                      "sample": f"C1 (configs/char_tower.yml shape, batch 64): {r1['steps']} steps in "
                                f"{r1['seconds']:.1f}s on {r1['threads']} threads"}}

    line = {
        "metric": "(query,doc) pairs/sec whole node at B=8192 d=256; HBM GB/s on embed gather",
        "value": round(value, 1),
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if scorer_dtype != "fp32" else "fp32",
        "data": "synthetic MS-MARCO-shaped id triplets (q 3-12 tokens, docs L/2-L), random-init weights",
        "config": {"workload": cfg["workload"] + (
                       f"; candidates all-gathered over ranks (C4, {'triplet form: M = N * 2B' if K == 1 else 'M = N * B'}"
                       f" = {M})" if world > 1 and cfg["loss"] == "in_batch" else ""),
                   "vocab": V, "d": d, "seq_len": L, "global_batch": B * world, "candidates_per_query": M,
                   "tokens_per_step_per_gpu": nnz, "parallelism": f"dp{world}", "scorer_dtype": scorer_dtype,
                   "table_sync": (tt.distributed.table_sync_mode(args.table_sync, E=d) if dp else "local"),
                   "hip_graph": use_graph, "graph_canary": canary,
                   "loop": (f"reference loop body unchanged (bench.PlainLoop, table_update {args.table_update})" if plain
                            else "TrainStep")},
        "gather_hbm_gbs": gather["achieved"] if gather else None,
        "gather_hbm": gather_hbm_evidence(args.config, gather, V, d),
        "roofline": roofline,
        # where the per-op times behind roofline / kernels come from: "graph_stamps" (a stamped
        # capture of the same step, replayed) or "eager_events_primed" (N ranks: an eager pass)
        "op_times": timing_source,
        "kernels": kernels,
        # the north_star's "B x B scorer at B=8192, d=256": M = B, the pairs form of this step
        "scorer_bxb": bxb,
        # the reference's train.py loop body unchanged around these registries (no TrainStep)
        "plain_loop": plain_entry,
        # N ranks: BASELINE configs[3] as stated (pairs form, M = N B; the main line is the triplet form)
        "c4_pairs": c4p,
        "cpu_baseline": cpu,
        "final_loss": float(loss.item()) if loss is not None else None,
    }
    print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
