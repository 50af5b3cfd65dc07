"""Cost of the two-launch data-parallel forward (tt_inbatch_fwd_ex_local + _remote) against the
one-launch tt_inbatch_fwd_ex on the same operands, on one GPU with nothing beside it (the rank
shapes of N = 2, 4, 8 at C4: B 8192 queries, 16384 own candidates, N x 16384 gathered).  The
difference is what splitting costs; what it hides (the candidate all-gather) needs the 8-GPU node."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from twotower_amd import _lib, ops  # noqa: E402
from twotower_amd._lib import call, ptr  # noqa: E402

dev = "cuda"
B, M, H, T, P = 8192, 16384, 256, _lib.TT_INBATCH_TAIL_ROWS, _lib.TT_INBATCH_MAX_PARTS
dt = _lib.compute_dtype_code("bf16")
g = torch.Generator(device=dev).manual_seed(0)
for N in (2, 4, 8):
    rank = N // 2
    q = torch.nn.functional.normalize(torch.randn(B, H, device=dev, generator=g), dim=-1)
    d_all = torch.nn.functional.normalize(torch.randn(N * M, H, device=dev, generator=g), dim=-1)
    st = torch.cuda.current_stream().cuda_stream
    qb = torch.empty(B + T, H, dtype=torch.bfloat16, device=dev)
    qn = torch.empty(B, device=dev)
    call("tt_inbatch_prep_rows", ptr(q), B, H, ptr(qb), ptr(qn), None, st)
    db_all = torch.zeros(N * M + T, H, dtype=torch.bfloat16, device=dev)
    parts_all = torch.zeros(N * P, device=dev)
    for r in range(N):
        call("tt_inbatch_prep_rows", ptr(d_all[r * M:(r + 1) * M]), M, H, ptr(db_all[r * M:]), None,
             ptr(parts_all[r * P:]), st)
    db = torch.zeros(M + T, H, dtype=torch.bfloat16, device=dev)
    db[:M] = db_all[rank * M:(rank + 1) * M]
    parts = parts_all[rank * P:(rank + 1) * P].clone()
    ws = torch.empty(_lib.lib().tt_inbatch_ex_ws_size(B, N * M, N * B, M, H, dt), dtype=torch.uint8, device=dev)
    lse, lse2, rows = (torch.empty(B, device=dev) for _ in range(3))
    loss = torch.empty((), device=dev)
    dqu = torch.empty(B, H, device=dev)

    def one():
        call("tt_inbatch_fwd_ex", ptr(qb), ptr(qn), B, ptr(db_all), ptr(parts_all), N * P, N * M, H, dt, 10.0,
             rank * M, 1, ptr(lse), ptr(lse2), ptr(rows), ptr(loss), ptr(dqu), ptr(ws), ws.numel(), st)

    def two():
        call("tt_inbatch_fwd_ex_local", ptr(qb), ptr(qn), B, ptr(db), ptr(parts), P, M, N * M, rank * M, H, dt,
             10.0, ptr(ws), ws.numel(), st)
        call("tt_inbatch_fwd_ex_remote", ptr(qb), ptr(qn), B, ptr(db_all), ptr(parts_all), N * P, ptr(parts), P, M,
             N * M, rank * M, H, dt, 10.0, 1, ptr(lse), ptr(lse2), ptr(rows), ptr(loss), ptr(dqu), ptr(ws),
             ws.numel(), st)

    res = {}
    for name, fn in (("one launch", one), ("two launches", two), ("one launch", one), ("two launches", two)):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) / 10 * 1e3
        out = (loss.item(), dqu.clone())
        res[name + " out"] = out
    a, b = res["one launch out"], res["two launches out"]
    err = ((a[1] - b[1]).abs().max() / a[1].abs().max()).item()
    print(f"N={N}: one launch {res['one launch']:.1f} us, two launches {res['two launches']:.1f} us "
          f"(loss {a[0]:.6f} vs {b[0]:.6f}, dq_unscaled rel {err:.1e})")
