"""Which host ops issue the device-to-device copies of the unchanged loop's step (torch.profiler,
the CPU op each memcpy belongs to).  Usage: python tools/repro/plain_memcpy.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402
import twotower_amd as tt  # noqa: E402

dev = torch.device("cuda")
cfg = bench.CONFIGS["c3"]
B, L, V = cfg["B"], cfg["L"], cfg["V"]
batches = [tt.data.synthetic_triplets(B, L, V, seed=100 + k, device=dev) for k in range(4)]
loss_fn = tt.losses.build("in_batch", temperature=0.1, compute_dtype="bf16")
_, model = bench.build_model(cfg, dev)
loop = bench.PlainLoop(model, loss_fn, table_update="backward_all")
for k in range(4):
    loop(*batches[k])
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    loop(*batches[0])
    torch.cuda.synchronize()
for e in prof.events():
    if "Memcpy" in e.name or "memcpy" in e.name.lower():
        chain, p = [], e.cpu_parent
        while p is not None:
            chain.append(p.name)
            p = p.cpu_parent
        print(e.name, round(e.device_time_total if hasattr(e, "device_time_total") else 0, 1), " <- ".join(chain[:6]),
              flush=True)
