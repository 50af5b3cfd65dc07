"""Which tensors tt_adamw_multi_ex changes differently from reduce + adamw_multi + prepare."""
import sys
sys.path.insert(0, ".")
import numpy as np
import torch
from twotower_amd import ops

DEV = "cuda"
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 96
rng = np.random.default_rng(7 + rows)
mats = [torch.as_tensor(rng.standard_normal((rows, 256)).astype(np.float32)).to(DEV) for _ in range(4)]
ws = ops.head_wgrad2(*mats)
shapes = [(256, 256), (256,), (256, 256), (256,)]
hyper = dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01)
runs = []
for fused in (False, True):
    r = np.random.default_rng(3)
    params = [[torch.as_tensor(r.standard_normal(s).astype(np.float32)).to(DEV) for _ in range(3)] for s in shapes]
    for p in params:
        p[2] = p[2].abs() * 0.01
    grads = [torch.full(s, float("nan"), device=DEV) for s in shapes]
    steps = [torch.full((), 4.0, device=DEV) for _ in range(4)]
    args = [torch.zeros(8, device=DEV) for _ in range(4)]
    slots = list(zip(steps, args))
    ops.adam_prepare(slots, increment=0, ahead=1, **hyper)
    args0 = [a.clone() for a in args]
    items = [(p, g, m, v, a) for (p, m, v), g, a in zip(params, grads, args)]
    if fused:
        sums = ops._Wgrad2Sums(ws, [p for p, _, _ in params]).grad_parts()
        ops.adamw_multi_ex(items, [sums[id(p)] for p, _, _ in params], slots,
                           ticket=torch.zeros(1, dtype=torch.int32, device=DEV), **hyper)
    else:
        ops.head_wgrad2_reduce(ws, *grads)
        ops.adamw_multi(items)
        ops.adam_prepare(slots, increment=1, ahead=1, **hyper)
    torch.cuda.synchronize()
    runs.append(([[t.clone() for t in it[:4]] for it in items], args0, [a.clone() for a in args]))
for k in range(4):
    for j, nm in enumerate("pgmv"):
        a, b = runs[0][0][k][j], runs[1][0][k][j]
        ne = (a != b) & ~(a.isnan() & b.isnan())
        print(k, nm, "equal" if not ne.any() else f"{int(ne.sum())} differ, max {float((a - b).abs().max()):.3e}, "
              f"first at {ne.nonzero()[0].tolist()}")
print("args before equal:", all(torch.equal(a, b) for a, b in zip(runs[0][1], runs[1][1])))
print("args after equal:", all(torch.equal(a, b) for a, b in zip(runs[0][2], runs[1][2])))
