"""Standalone time of the bag backward sort plan (tt_bag_plan) at the bench shape, graph-replayed."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import twotower_amd as tt
from twotower_amd import ops

# shape: c3 (default: 3 x 8192 sequences of 64 ids over 200k rows) or c5 (6 x 8192 over 1M rows)
shape = sys.argv[1] if len(sys.argv) > 1 else "c3"
B, L, V, E = 8192, 64, (1_000_000 if shape == "c5" else 200_000), 256
K = 4 if shape == "c5" else 1
idsets = {}
for name, z in (("uniform", None), ("zipf1.0", 1.0)):
    parts = tt.data.synthetic_triplets(B, L, V, seed=0, device="cuda", zipf_s=z, negatives=K)
    idsets[name] = torch.cat(list(parts)).to(torch.int32).contiguous()


def t(fn, it=10, reps=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(it):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (it * reps) * 1e3


for name, ids in idsets.items():
    def plan():
        pl = ops.BagPlan(ids, V, E, 0)
        pl.wait()
    print(f"tt_bag_plan {shape} {name} maxd {os.environ.get('TT_PLAN_MAXD', 'default')}: {t(plan):.1f} us")
