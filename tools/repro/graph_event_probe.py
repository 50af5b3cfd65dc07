"""Probe: HIP events recorded INSIDE a captured graph (torch.cuda.Event(external=True) -> event
record nodes) time a kernel of the replayed graph.  Compares with eager event timing of the same op."""
import torch

a = torch.randn(4096, 4096, device="cuda")
b = torch.randn(4096, 4096, device="cuda")
torch.cuda.synchronize()
e0 = torch.cuda.Event(enable_timing=True, external=True)
e1 = torch.cuda.Event(enable_timing=True, external=True)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(2):
        c = a @ b
        d = c @ b
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    c = a @ b
    e0.record()
    d = c @ b
    e1.record()
for i in range(5):
    g.replay()
    torch.cuda.synchronize()
    print("graph replay", i, "second matmul ms", round(e0.elapsed_time(e1), 4), flush=True)
x0, x1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for i in range(3):
    c = a @ b
    x0.record()
    d = c @ b
    x1.record()
    torch.cuda.synchronize()
    print("eager", i, round(x0.elapsed_time(x1), 4), flush=True)
print("probe ok")
