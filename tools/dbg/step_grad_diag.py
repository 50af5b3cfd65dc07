"""Where do the HIP step gradients differ from float64?  At a given shape: the HIP plain autograd
path, the HIP TrainStep path (lr 0: parameters unchanged, tower gradients left in .grad), ATen
fp32 and float64 restatements of the reference step (oracle/cpu_step.py's tower on the GPU), each
parameter's max-normalised error against float64, plus the count of hidden pre-activations
within fp32 rounding of zero (ReLU decisions that may legitimately flip).
Usage: python tools/dbg/step_grad_diag.py [V E L B K loss]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import torch  # noqa: E402

import twotower_amd as tt  # noqa: E402
import _step_parity as sp  # noqa: E402
from oracle.cpu_step import RefTower  # noqa: E402

a = sys.argv[1:]
V, E, L, B, K = (int(x) for x in (a[:5] if len(a) >= 5 else (3000, 256, 24, 48, 4)))
loss_name = a[5] if len(a) > 5 else "multiple_negatives"
DEV = "cuda"
torch.manual_seed(11)
emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
model = tt.build_two_tower("mean", emb, hidden_dim=E, tied_weights=True).to(DEV)
init = {k: v.detach().clone() for k, v in model.named_parameters()}
batch = tt.data.synthetic_triplets(B, L, V, seed=111, device=DEV, negatives=K)
hip_loss = sp._hip_loss(loss_name, "fp32", K)

q, p, n = model(*batch)
lh = hip_loss(q, p, n)
lh.backward()
g_plain = {k: v.grad.detach().clone() for k, v in model.named_parameters()}
model.zero_grad(set_to_none=True)

opt = tt.optim.AdamW(model.parameters(), lr=0.0, weight_decay=0.0, fused_tables=True, tables=[emb], capturable=True)
step = tt.TrainStep(model, hip_loss, opt)
step(*batch)
torch.cuda.synchronize()
g_step = {k: (v.grad.detach().clone() if v.grad is not None else None) for k, v in model.named_parameters()}


def ref_grads(dtype):
    ref = RefTower(V, E, E).to(dtype).to(DEV)
    ref.load_state_dict({sp._ref_key(k): v.to(dtype) for k, v in init.items()})
    ids = [t.long() for t in batch]
    outs = [ref(t) for t in ids]
    sp._loss64(loss_name, *outs, K).backward()
    sd = ref.state_dict(keep_vars=True)
    x = ref.embedding(ids[0]).sum(1)  # noqa: F841
    return {k: sd[sp._ref_key(k)].grad for k in init}, ref


g64, ref64 = ref_grads(torch.float64)
g32, _ = ref_grads(torch.float32)
for k in init:
    line = [k.split(".")[-2] + "." + k.split(".")[-1]]
    for nm, g in (("plain", g_plain.get(k)), ("step", g_step.get(k)), ("aten32", g32[k])):
        line.append(f"{nm} {sp._rel(g, g64[k]):.2e}" if g is not None else f"{nm} -")
    print("  ".join(line), flush=True)
with torch.no_grad():
    ids = torch.cat([t.long() for t in batch])
    m = (ids > 0).double().unsqueeze(-1)
    pooled = (ref64.embedding(ids) * m).sum(1) / (m.sum(1) + 1e-9)
    h = pooled @ ref64.feed_forward[0].weight.T + ref64.feed_forward[0].bias
    tiny = (h.abs() < 1e-6 * h.abs().max()).sum().item()
    print(f"pre-activations within 1e-6 of max|h| of zero: {tiny} of {h.numel()}; exact zeros {(h == 0).sum().item()}")
