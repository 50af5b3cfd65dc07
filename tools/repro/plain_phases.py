"""Host time to issue each phase of the unchanged train.py loop body at C3 (bench.PlainLoop with
both config opt-ins), no host syncs inside the timed steps: model forward, loss, zero_grad,
backward (the autograd engine's thread included), optimizer.step.  Usage:
python tools/repro/plain_phases.py [steps] [mode]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import twotower_amd as tt  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
mode = sys.argv[2] if len(sys.argv) > 2 else "backward_all"
dev = torch.device("cuda")
cfg = bench.CONFIGS["c3"]
B, L, V = cfg["B"], cfg["L"], cfg["V"]
batches = [tt.data.synthetic_triplets(B, L, V, seed=100 + k, device=dev) for k in range(4)]
loss_fn = tt.losses.build("in_batch", temperature=0.1, compute_dtype="bf16")
_, model = bench.build_model(cfg, dev)
loop = bench.PlainLoop(model, loss_fn, table_update=mode)
opt = loop.optimizer
acc = {k: 0.0 for k in ("forward", "loss", "zero_grad", "backward", "step")}
for k in range(steps + 5):
    q, p, n = batches[k % 4]
    t0 = time.perf_counter()
    outs = model(q, p, n)
    t1 = time.perf_counter()
    loss = loss_fn(*outs)
    t2 = time.perf_counter()
    opt.zero_grad()
    t3 = time.perf_counter()
    loss.backward()
    t4 = time.perf_counter()
    opt.step()
    t5 = time.perf_counter()
    if k >= 5:
        for key, a, b in (("forward", t0, t1), ("loss", t1, t2), ("zero_grad", t2, t3), ("backward", t3, t4),
                          ("step", t4, t5)):
            acc[key] += (b - a) * 1e3
    if k % 4 == 3:
        torch.cuda.synchronize()  # keep the queue from running far ahead (every 4 steps, outside the phases)
torch.cuda.synchronize()
print({k: round(v / steps, 4) for k, v in acc.items()}, "total", round(sum(acc.values()) / steps, 4), flush=True)
