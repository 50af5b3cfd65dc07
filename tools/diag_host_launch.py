"""Diagnostic (GPU, not a test): is the replayed C3 step host-bound?

Times (a) the host's enqueue cost per step (torch.cat into the static buffer + graph.replay(),
no sync), (b) the device time per step with K steps enqueued back to back, (c) a single replay
in isolation (sync before and after).  If (a) >= (b) the GPU waits for the host.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import twotower_amd as tt  # noqa: E402

V, d, L, B = 200_000, 256, 64, 8192
dev = torch.device("cuda", 0)
torch.manual_seed(1234)
emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=d)
model = tt.build_two_tower("mean", emb, hidden_dim=d, tied_weights=True).to(dev)
loss_fn = tt.losses.build("in_batch", temperature=0.1, compute_dtype="bf16")
opt = tt.optim.AdamW(model.parameters(), lr=1e-3, fused_tables=True, tables=[emb], capturable=True)
step = tt.TrainStep(model, loss_fn, opt, graph=True)
batches = [tt.data.synthetic_triplets(B, L, V, seed=k, device=dev) for k in range(4)]
for k in range(6):
    step(*batches[k % 4])
torch.cuda.synchronize()
graph, static_all, _ = next(iter(step._graphs.values()))
print("graph nodes:", getattr(graph, "num_nodes", lambda: "?")() if hasattr(graph, "num_nodes") else "?")

K = 30
host = []
t0 = time.perf_counter()
for k in range(K):
    h0 = time.perf_counter()
    step(*batches[k % 4])
    host.append(time.perf_counter() - h0)
h_end = time.perf_counter()
torch.cuda.synchronize()
t1 = time.perf_counter()
print(f"enqueue per step: mean {1e3 * sum(host) / K:.3f} ms, min {1e3 * min(host):.3f} ms; "
      f"host loop {1e3 * (h_end - t0) / K:.3f} ms/step; wall {1e3 * (t1 - t0) / K:.3f} ms/step")

single = []
for k in range(10):
    torch.cuda.synchronize()
    s0 = time.perf_counter()
    step(*batches[k % 4])
    torch.cuda.synchronize()
    single.append(time.perf_counter() - s0)
print(f"isolated step (sync both sides): min {1e3 * min(single):.3f} ms, mean {1e3 * sum(single) / 10:.3f} ms")

# replay only (no cat)
torch.cuda.synchronize()
s0 = time.perf_counter()
for k in range(K):
    graph.replay()
r_host = time.perf_counter() - s0
torch.cuda.synchronize()
s1 = time.perf_counter()
print(f"replay-only: host {1e3 * r_host / K:.3f} ms/step, wall {1e3 * (s1 - s0) / K:.3f} ms/step")
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record()
for k in range(K):
    graph.replay()
ev[1].record()
torch.cuda.synchronize()
print(f"replay-only events: {ev[0].elapsed_time(ev[1]) / K:.3f} ms/step")
