"""B x B scorer timeline (M = B = 8192, H = 256, bf16): where the forward + backward time goes.

The sequence is the one TrainStep runs for the pairs form (`bench.py` scorer_bxb): the operand prep in
the head's normalise pass (tt_inbatch_l2_prep), the forward (tt_inbatch_fwd_prepped) and the backward
fused with F.normalize's backward (tt_inbatch_bwd_l2), captured in one HIP graph and replayed.

Two runs make the timeline:
  * `python tools/bxb_timeline.py run`      under `rocprofv3 --kernel-trace` (normal library): each
    kernel's start / end per replay -> per-kernel durations and the gaps between them;
  * `python tools/bxb_timeline.py ktrace LIB` with a TT_SCORER_TRACE variant library: per-workgroup
    s_memrealtime at engine entry / loop start / loop end / exit -> prologue, loop, epilogue and the
    slowest-XCD tail of each engine.
  * `python tools/bxb_timeline.py report KERNEL_TRACE_CSV [KTRACE_TXT]` prints the table.
"""
import csv
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

B = M = 8192
H = 256


def setup():
    import torch
    from twotower_amd import _lib
    from twotower_amd._lib import call, ptr

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    x0 = torch.randn(B + M, H, device=dev, generator=g)
    qd = torch.empty_like(x0)
    norms = torch.empty(B + M, device=dev)
    dt = _lib.TT_BF16
    nbytes = _lib.lib().tt_inbatch_ws_size(B, M, H, dt)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    lse = torch.empty(B, device=dev)
    rows = torch.empty(B, device=dev)
    loss = torch.empty((), device=dev)
    dqu = torch.empty(B, H, device=dev)
    gs = torch.ones(1, device=dev)
    dx = torch.empty_like(qd)
    inv_tau = 10.0

    def seq():
        s = torch.cuda.current_stream(dev).cuda_stream
        qd.copy_(x0)
        call("tt_inbatch_l2_prep", ptr(qd), B, M, H, dt, ptr(norms), ptr(ws), ws.numel(), s)
        call("tt_inbatch_fwd_prepped", ptr(qd), ptr(qd[B:]), B, M, H, dt, inv_tau, 0, 1, ptr(lse), ptr(rows), None,
             ptr(dqu), ptr(ws), ws.numel(), s)
        call("tt_inbatch_bwd_l2", ptr(qd), B, M, H, dt, inv_tau, 0, ptr(lse), ptr(dqu), ptr(gs), 1.0 / B, ptr(norms),
             ptr(dx), ptr(rows), ptr(loss), ptr(ws), ws.numel(), s)

    return torch, dev, seq, loss


def run(reps: int = 30):
    torch, dev, seq, loss = setup()
    for _ in range(3):
        seq()
    torch.cuda.synchronize()
    st = torch.cuda.Stream(dev)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.stream(st):
        seq()  # warm the capture stream
        torch.cuda.synchronize()
        with torch.cuda.graph(gr, stream=st):
            seq()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(5):
        gr.replay()
    torch.cuda.synchronize()
    t0.record()
    for _ in range(reps):
        gr.replay()
    t1.record()
    torch.cuda.synchronize()
    print(json.dumps({"bxb_graph_us_per_replay": round(t0.elapsed_time(t1) * 1e3 / reps, 2), "loss": float(loss)}))


def ktrace(libpath: str):
    if libpath:
        from twotower_amd import _lib
        _lib.LIB_PATH = os.path.abspath(libpath)
    torch, dev, seq, _ = setup()
    import numpy as np
    from twotower_amd import _lib
    for _ in range(4):
        seq()
    torch.cuda.synchronize()
    kb = (ctypes.c_longlong * 8192)()
    fk = _lib.lib().tt_debug_scorer_ktrace
    fk.argtypes, fk.restype = [ctypes.c_void_p], ctypes.c_int
    fk(kb)
    out = {}
    for which, base in (("backward", 0), ("forward", 4096)):
        k = np.array(kb[base:base + 4096], dtype=np.int64).reshape(1024, 4)
        idx = np.nonzero(k[:, 0] > 0)[0]
        k = k[idx]
        if not len(k):
            continue
        t0 = k[:, 0].min()
        us = (k - t0) / 100.0  # 100 MHz ticks -> us
        xcd = idx % 8
        loop = us[:, 2] - us[:, 1]
        rec = {
            "workgroups": int(len(k)),
            "entry_max_us": float(us[:, 0].max()),
            "prologue_med_us": float(np.median(us[:, 1] - us[:, 0])),
            "loop_start_med_us": float(np.median(us[:, 1])),
            "loop_med_us": float(np.median(loop)),
            "loop_min_us": float(loop.min()),
            "loop_max_us": float(loop.max()),
            "epilogue_med_us": float(np.median(us[:, 3] - us[:, 2])),
            "exit_med_us": float(np.median(us[:, 3])),
            "exit_max_us": float(us[:, 3].max()),
            "tail_us": float(us[:, 3].max() - np.median(us[:, 3])),
            "loop_med_by_xcd": [round(float(np.median(loop[xcd == x])), 2) for x in range(8)],
            "exit_max_by_xcd": [round(float(us[xcd == x, 3].max()), 2) for x in range(8)],
        }
        out[which] = rec
        print(which, json.dumps(rec))
    return out


def _kernels(path: str):
    """(start ns, end ns, name) of every dispatch in a rocprofv3 kernel trace: the rocpd SQLite
    database (rocprofv3's default output) or a kernel_trace.csv."""
    if path.endswith(".db"):
        import sqlite3
        c = sqlite3.connect(path)
        return sorted((int(s), int(e), n) for n, s, e in c.execute("select name, start, end from kernels"))
    ks = []
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name") or r.get("KernelName") or ""
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    return sorted(ks)


def report(csv_path: str, ktrace_path: str | None = None):
    ks = _kernels(csv_path)
    # a replay = the kernels from one l2_prep launch to the next
    ks = [k for k in ks if "copyBuffer" not in k[2]]  # the graph's input refresh (qd.copy_)
    starts = [i for i, k in enumerate(ks) if "l2_prep" in k[2]]
    reps = [ks[starts[i]:starts[i + 1]] for i in range(len(starts) - 1)]
    reps = reps[len(reps) // 3:]  # drop warmup / first-call replays
    import numpy as np

    def short(n):
        for key in ("l2_prep", "score_bf16", "fwd_combine", "score_ddp", "bwd_combine_l2", "bwd_combine", "mean"):
            if key in n:
                return key
        return n.split("(")[0][-40:]

    names = [short(k[2]) for k in reps[0]]
    dur = np.array([[(k[1] - k[0]) / 1e3 for k in r] for r in reps if len(r) == len(names)])
    gap = np.array([[(r[i + 1][0] - r[i][1]) / 1e3 for i in range(len(r) - 1)] for r in reps if len(r) == len(names)])
    span = np.array([(r[-1][1] - r[0][0]) / 1e3 for r in reps if len(r) == len(names)])
    print(f"B x B scorer timeline, {len(dur)} replays (median us)")
    for i, n in enumerate(names):
        g = f"  gap after {np.median(gap[:, i]):6.2f}" if i < len(names) - 1 else ""
        print(f"  {n:22s} {np.median(dur[:, i]):8.2f}{g}")
    print(f"  span l2_prep start -> last end {np.median(span):8.2f}")
    if ktrace_path:
        print(open(ktrace_path).read())


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "run"
    if what == "run":
        run()
    elif what == "ktrace":
        ktrace(sys.argv[2] if len(sys.argv) > 2 else "")
    else:
        report(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
