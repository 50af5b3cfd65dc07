"""One rank's scorer work under data parallelism with cross-device negatives (candidate-owner
gradients), simulated on one GPU: tt_inbatch_fwd_ex over this rank's B queries x all W * M
candidates, tt_inbatch_bwd_ex over this rank's M candidates x all W * B queries (the buffers
the all-gathers would fill are synthetic).  Prints per-pass us and executed TFLOP/s
(4 * B * W * M * H per pass) for W = 1, 2, 4, 8 at the C3/C4 shape (B 8192, M 2B, H 256)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from twotower_amd import _lib  # noqa: E402

B, H, T, P = 8192, 256, _lib.TT_INBATCH_TAIL_ROWS, _lib.TT_INBATCH_MAX_PARTS
M = 2 * B
dt = _lib.compute_dtype_code(sys.argv[1] if len(sys.argv) > 1 else "bf16")
st = torch.cuda.current_stream().cuda_stream
g = torch.Generator(device="cuda").manual_seed(0)


def unit(n):
    return torch.nn.functional.normalize(torch.randn(n, H, device="cuda", generator=g), dim=-1)


def timed(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


for W in (1, 2, 4, 8):
    q, d_all, q_all = unit(B), unit(W * M), unit(W * B)
    qb = torch.empty(B + T, H, dtype=torch.bfloat16, device="cuda")
    qn = torch.empty(B, device="cuda")
    _lib.call("tt_inbatch_prep_rows", q.data_ptr(), B, H, qb.data_ptr(), qn.data_ptr(), None, st)
    db_all = torch.empty(W * M + T, H, dtype=torch.bfloat16, device="cuda")
    parts = torch.empty(P, device="cuda")
    _lib.call("tt_inbatch_prep_rows", d_all.data_ptr(), W * M, H, db_all.data_ptr(), None, parts.data_ptr(), st)
    qb_all = torch.empty(W * B + T, H, dtype=torch.bfloat16, device="cuda")
    _lib.call("tt_inbatch_prep_rows", q_all.data_ptr(), W * B, H, qb_all.data_ptr(), None, None, st)
    db = db_all[:M + T]  # this rank's candidates (rank 0), zero tail not needed by the backward
    ws = torch.empty(_lib.lib().tt_inbatch_ex_ws_size(B, W * M, W * B, M, H, dt), dtype=torch.uint8, device="cuda")
    lse, lse2, rows = (torch.empty(B, device="cuda") for _ in range(3))
    loss = torch.empty((), device="cuda")
    dqu, dq, dd = torch.empty(B, H, device="cuda"), torch.empty(B, H, device="cuda"), torch.empty(M, H, device="cuda")
    lse2_all = torch.empty(W * B + T, device="cuda")
    gl = torch.ones(1, device="cuda")

    def fwd():
        _lib.call("tt_inbatch_fwd_ex", qb.data_ptr(), qn.data_ptr(), B, db_all.data_ptr(), parts.data_ptr(), P,
                  W * M, H, dt, 10.0, 0, 1, lse.data_ptr(), lse2.data_ptr(), rows.data_ptr(), loss.data_ptr(),
                  dqu.data_ptr(), ws.data_ptr(), ws.numel(), st)

    fwd()
    lse2_all[:W * B] = lse2.repeat(W)
    lse2_all[W * B:] = float("inf")

    def bwd():
        _lib.call("tt_inbatch_bwd_ex", qb_all.data_ptr(), lse2_all.data_ptr(), W * B, 0, db.data_ptr(), M, B, 0, H, dt,
                  10.0, dqu.data_ptr(), gl.data_ptr(), 1.0 / B, dq.data_ptr(), dd.data_ptr(), ws.data_ptr(),
                  ws.numel(), st)

    tf, tb = timed(fwd), timed(bwd)
    fl = 4.0 * B * W * M * H
    print(json.dumps({"world": W, "candidates": W * M, "fwd_us": round(tf, 1), "bwd_us": round(tb, 1),
                      "fwd_tflops": round(fl / tf / 1e6, 1), "bwd_tflops": round(fl / tb / 1e6, 1)}), flush=True)
