"""Debug: gather-mode DP step vs single-process step (2 ranks gloo on one GPU)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.distributed as dist
import twotower_amd as tt

rank = int(os.environ["RANK"]); world = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("gloo")
V, E, B, L = 3001, 64, 64, 24
LR = 1e6


def build(w, sync):
    torch.manual_seed(7)
    emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
    model = tt.build_two_tower("mean", emb, hidden_dim=E, tied_weights=True).to("cuda:0")
    opt = tt.optim.AdamW(model.parameters(), lr=LR, eps=1.0, weight_decay=0.0, fused_tables=True, tables=[emb],
                         capturable=True, table_sync=sync, group=None)
    return model, emb, tt.TrainStep(model, tt.losses.build("triplet", margin=0.2), opt)

full = tt.data.synthetic_triplets(world * B, L, V, seed=3, device="cuda:0")
# single-process reference computed on every rank without DP: use a subgroup trick -> build before DP is visible
model, emb, step = build(world, "gather")
w0 = emb.weight.detach().clone()
b = tuple(t[rank * B:(rank + 1) * B] for t in full)
step(*b)
torch.cuda.synchronize()
d = (emb.weight.detach() - w0)
dl = [torch.empty_like(d) for _ in range(world)]
dist.all_gather(dl, d)
print(rank, "ranks agree:", torch.equal(dl[0], dl[1]), flush=True)
touched = torch.zeros(V, dtype=torch.bool, device="cuda:0")
for r in range(world):
    ids = torch.cat([t[r * B:(r + 1) * B] for t in full]).long().flatten()
    m = torch.zeros(V, dtype=torch.bool, device="cuda:0"); m[ids] = True
    print(rank, f"rows touched by rank{r}:", int(m.sum()), "changed rows among them:", int((d.abs().sum(1) > 0)[m].sum()), flush=True)
    touched |= m
print(rank, "changed rows not touched:", int(((d.abs().sum(1) > 0) & ~touched).sum()), flush=True)
dist.destroy_process_group()
