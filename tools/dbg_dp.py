"""Debug the gather-mode DP table update: 2 ranks on one GPU over gloo."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.distributed as dist
import twotower_amd as tt
from twotower_amd import ops

rank = int(os.environ["RANK"]); world = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("gloo")
V, E, B, L = 3001, 64, 64, 24
full = tt.data.synthetic_triplets(world * B, L, V, seed=3, device="cuda:0")
ids = torch.cat([t[rank * B:(rank + 1) * B] for t in full], 0).contiguous()
plan = ops.BagPlan(ids, V, E, 0, gather_group=dist.group.WORLD)
plan.wait()
torch.cuda.synchronize()
exp = torch.cat([torch.cat([t[r * B:(r + 1) * B] for t in full], 0) for r in range(world)], 0)
print(rank, "ids_all equal:", torch.equal(plan.ids, exp), plan.ids.shape, flush=True)
# compare planned dense grads: gathered plan vs local plan on the concatenated ids
dp = torch.randn(world * 3 * B, E, device="cuda:0", generator=torch.Generator("cuda").manual_seed(1))
den = torch.rand(world * 3 * B, device="cuda:0", generator=torch.Generator("cuda").manual_seed(2)) + 1
g1 = ops.bag_mean_backward_planned(dp, den, plan)
g2 = ops.bag_mean_backward(dp, den, exp, V, 0)
print(rank, "grad equal:", torch.equal(g1, g2), (g1 - g2).abs().max().item(), flush=True)
dist.destroy_process_group()
