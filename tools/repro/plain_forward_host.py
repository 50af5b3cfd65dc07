"""Host time from the start of the reference loop's step (bench.PlainLoop, both opt-ins) to the
launch of its bag gather, i.e. the GPU's idle time at the start of a step that follows the loop's
.item() syncs.  Usage: python tools/repro/plain_forward_host.py [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import twotower_amd as tt  # noqa: E402
from twotower_amd import _lib  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
dev = torch.device("cuda")
cfg = bench.CONFIGS["c3"]
B, L, V = cfg["B"], cfg["L"], cfg["V"]
batches = [tt.data.synthetic_triplets(B, L, V, seed=100 + k, device=dev) for k in range(4)]
loss_fn = tt.losses.build("in_batch", temperature=0.1, compute_dtype="bf16")
_, model = bench.build_model(cfg, dev)
loop = bench.PlainLoop(model, loss_fn, table_update="backward_all")
marks = {}
orig = _lib.call


def call(name, *args):
    if name not in marks:
        marks[name] = time.perf_counter()
    return orig(name, *args)


for k in range(5):
    loop(*batches[k % 4])
torch.cuda.synchronize()
res = {}
for k in range(steps):
    _lib.call = call
    import twotower_amd.ops as ops_mod
    ops_mod.call = call
    marks.clear()
    t0 = time.perf_counter()
    outs = model(*batches[k % 4])
    t1 = time.perf_counter()
    ops_mod.call = orig
    _lib.call = orig
    loss = loop.loss_fn(*outs)
    loop.optimizer.zero_grad()
    loss.backward()
    loop.optimizer.step()
    loss.item()
    for n, t in marks.items():
        res.setdefault(n, []).append((t - t0) * 1e6)
    res.setdefault("forward_total", []).append((t1 - t0) * 1e6)
for n, v in sorted(res.items(), key=lambda kv: sorted(kv[1])[len(kv[1]) // 2]):
    v = sorted(v)
    print(f"{n}: median {v[len(v) // 2]:.1f} us after the step's start (min {v[0]:.1f})")

# where the forward's host time goes (cProfile over the same steps' model() calls)
if len(sys.argv) > 2 and sys.argv[2] == "profile":
    import cProfile
    import pstats
    pr = cProfile.Profile()
    for k in range(steps):
        pr.enable()
        outs = model(*batches[k % 4])
        pr.disable()
        loss = loop.loss_fn(*outs)
        loop.optimizer.zero_grad()
        loss.backward()
        loop.optimizer.step()
        loss.item()
    st = pstats.Stats(pr)
    st.sort_stats("cumulative").print_stats(40)
    st.sort_stats("tottime").print_stats(30)
