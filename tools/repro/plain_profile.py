"""Where the unchanged train.py loop (bench.PlainLoop, table_update "backward") spends its step at C3.

Times the loop as is and with parts removed (monitors, optimizer step), and prints torch.profiler's
per-op CPU / GPU totals over a few steps plus the GPU-busy fraction of the step (sum of kernel
times / wall).  Usage: python tools/repro/plain_profile.py [steps] [optimizer|backward|backward_all]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import twotower_amd as tt  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda")
cfg = bench.CONFIGS["c3"]
B, L, V, K = cfg["B"], cfg["L"], cfg["V"], cfg.get("K", 1)
batches = [tt.data.synthetic_triplets(B, L, V, seed=100 + k, device=dev) for k in range(4)]
loss_fn = tt.losses.build("in_batch", temperature=0.1, compute_dtype="bf16")
_, model = bench.build_model(cfg, dev)
mode = sys.argv[2] if len(sys.argv) > 2 else "backward"
loop = bench.PlainLoop(model, loss_fn, table_update=mode)


def no_monitor(q, p, n):
    outs = model(q, p, n)
    loss = loop.loss_fn(*outs)
    loop.optimizer.zero_grad()
    loss.backward()
    loop.optimizer.step()
    return loss


def no_step(q, p, n):
    outs = model(q, p, n)
    loss = loop.loss_fn(*outs)
    loop.optimizer.zero_grad()
    loss.backward()
    return loss


def fwd_only(q, p, n):
    with torch.no_grad():
        outs = model(q, p, n)
        return loop.loss_fn(*outs)


res = {}
for name, fn in (("loop", loop), ("no_monitors", no_monitor), ("no_optimizer_step", no_step), ("forward_loss_nograd", fwd_only)):
    res[name] = round(bench.time_steps(fn, batches, steps, 3), 4)
print({"ms_per_step": res}, flush=True)

# CPU launch time of one step with the GPU kept busy: queue a long sleep first so no sync stalls
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(steps):
    no_monitor(*batches[k % 4])
t_cpu = (time.perf_counter() - t0) / steps * 1e3
torch.cuda.synchronize()
print({"cpu_issue_ms_per_step_no_monitors": round(t_cpu, 4)}, flush=True)

from torch.profiler import ProfilerActivity, profile  # noqa: E402

with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    for k in range(3):
        loop(*batches[k % 4])
    torch.cuda.synchronize()
ka = prof.key_averages()
print(ka.table(sort_by="cpu_time_total", row_limit=30), flush=True)
print(ka.table(sort_by="device_time_total", row_limit=25), flush=True)
gpu_us = sum(e.self_device_time_total for e in ka if e.device_type is not None and str(e.device_type).endswith("CUDA"))
print({"gpu_kernel_us_per_step": round(gpu_us / 3, 1)}, flush=True)

# Python-side cost of issuing a step (no monitors: no host syncs), by function
import cProfile  # noqa: E402
import pstats  # noqa: E402

torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for k in range(steps):
    no_monitor(*batches[k % 4])
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(45)
st.sort_stats("cumulative").print_stats(45)
