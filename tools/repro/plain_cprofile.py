"""cProfile of the host side of the unchanged loop's forward and backward at C3 (bench.PlainLoop,
both opt-ins), many iterations so per-function host costs resolve.  Usage:
python tools/repro/plain_cprofile.py [iters]"""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import twotower_amd as tt  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 100
dev = torch.device("cuda")
cfg = bench.CONFIGS["c3"]
B, L, V = cfg["B"], cfg["L"], cfg["V"]
batches = [tt.data.synthetic_triplets(B, L, V, seed=100 + k, device=dev) for k in range(4)]
loss_fn = tt.losses.build("in_batch", temperature=0.1, compute_dtype="bf16")
_, model = bench.build_model(cfg, dev)
loop = bench.PlainLoop(model, loss_fn, table_update="backward_all")
opt = loop.optimizer


def body(k):
    outs = model(*batches[k % 4])
    loss = loss_fn(*outs)
    opt.zero_grad()
    loss.backward()
    opt.step()


for k in range(5):
    body(k)
torch.cuda.synchronize()
# the autograd engine runs backward on its own thread: profile that thread too
import threading  # noqa: E402

prof = cProfile.Profile()
threading.setprofile(lambda *a: None)
torch.autograd.set_multithreading_enabled(False)  # backward on this thread, so cProfile sees it
prof.enable()
for k in range(iters):
    body(k)
    if k % 4 == 3:
        torch.cuda.synchronize()
prof.disable()
torch.cuda.synchronize()
st = pstats.Stats(prof)
st.sort_stats("tottime").print_stats(40)
