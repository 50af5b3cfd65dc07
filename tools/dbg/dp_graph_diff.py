"""Eager vs graph N-rank step (one forced RCCL rank, shard exchange): after N steps, which
parameters / optimizer state differ, and for the table which rows (touched by the last batch or
not, own chunk position).  Usage: python tools/dbg/dp_graph_diff.py [steps] [table_sync]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["TT_DIST_FORCE"] = "1"
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29641")
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import twotower_amd as tt  # noqa: E402

nsteps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
table_sync = sys.argv[2] if len(sys.argv) > 2 else "shard"
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
V, E, L, B = 3000, 256, 16, 256
batches = [tt.data.synthetic_triplets(B, L, V, seed=s, device="cuda") for s in range(4)]
res = {}
for graph in (False, True):
    torch.manual_seed(0)
    emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
    model = tt.build_two_tower("mean", emb, hidden_dim=E, tied_weights=True).cuda()
    loss_fn = tt.losses.build("in_batch", temperature=0.1, compute_dtype="bf16", cross_device_negatives=True)
    opt = tt.optim.AdamW(model.parameters(), lr=1e-3, fused_tables=True, tables=[emb], capturable=True,
                         table_sync=table_sync)
    step = tt.TrainStep(model, loss_fn, opt, graph=graph, eager_steps=1)
    for s in range(nsteps):
        step(*batches[s % 4])
    torch.cuda.synchronize()
    st = {}
    for k, p in model.named_parameters():
        st[k] = p.detach().clone()
        for sk, sv in opt.state[p].items():
            if torch.is_tensor(sv):
                st[k + "/" + sk] = sv.detach().clone()
    res[graph] = st
out = {}
for k in res[False]:
    a, b = res[False][k], res[True][k]
    if a.shape != b.shape:
        out[k] = f"shape {tuple(a.shape)} vs {tuple(b.shape)}"
        continue
    d = (a.double() - b.double()).abs()
    if d.max() > 0:
        info = {"max": float(d.max()), "n": int((d > 0).sum())}
        if d.dim() == 2:
            rows = (d.max(1).values > 0).nonzero().flatten()
            info["rows"] = int(rows.numel())
            last = torch.cat([t.reshape(-1) for t in batches[(nsteps - 1) % 4]]).unique()
            info["rows_in_last_batch"] = int(torch.isin(rows, last).sum())
            info["first_rows"] = rows[:8].tolist()
        if d.dim() <= 1 and d.numel() <= 4:
            info["values"] = [a.tolist(), b.tolist()]
        out[k] = info
print(json.dumps(out, indent=1), flush=True)
dist.destroy_process_group()
