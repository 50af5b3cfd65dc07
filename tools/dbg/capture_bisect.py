"""Where does capturing the data-parallel step segfault?  One forced nccl rank (world 1), the
bench's DP TrainStep objects warmed up by one eager step, then ONE capture of a growing prefix:

  fwd        model forward + cross-device loss forward
  fwd_bwd    + loss.backward (the autograd thread's collectives)
  full       + optimizer.step (table exchange, gradient all-reduce on the comm stream)

Usage: python tools/dbg/capture_bisect.py MODE [gather|shard] [local]   ('local': no
cross-device negatives).  Prints one JSON line if the capture ends."""
import faulthandler
import json
import os
import sys

faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["TT_DIST_FORCE"] = "1"
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29537")
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import twotower_amd as tt  # noqa: E402
from twotower_amd import ops  # noqa: E402

mode = sys.argv[1]
sync = sys.argv[2] if len(sys.argv) > 2 else "gather"
xdev = not (len(sys.argv) > 3 and sys.argv[3] == "local")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
torch.cuda.set_device(0)
torch.manual_seed(0)
emb = tt.embeddings.build("lookup", vocab_size=5000, embedding_dim=128)
model = tt.build_two_tower("mean", emb, hidden_dim=128, tied_weights=True).cuda()
loss_fn = tt.losses.build("in_batch", temperature=0.1, compute_dtype="fp32", cross_device_negatives=xdev)
opt = tt.optim.AdamW(model.parameters(), fused_tables=True, tables=[emb], capturable=True, table_sync=sync)
step = tt.TrainStep(model, loss_fn, opt, graph=False)
batch = tt.data.synthetic_triplets(256, 16, 5000, seed=1, device="cuda")
for _ in range(int(os.environ.get("TT_BISECT_WARMUP", "1"))):
    first = float(step.eager(*batch))
torch.cuda.synchronize()
print(f"eager step ok: loss {first:.6f}", flush=True)

side = getattr(opt, "_side_grads", None)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    if side is not None:
        side.join()
        side.active = True
    with ops.deferred_loss_mean(), step._scorer_prep_open():
        loss = loss_fn(*model(*batch))
    if mode in ("fwd_bwd", "full"):
        opt.zero_grad(set_to_none=True)
        seed = torch.full((), step.sync.loss_scale() if step.sync is not None else 1.0, device="cuda")
        with ops.uniform_loss_seed(), ops.fused_head_backward():
            loss.backward(seed)
    if mode == "full":
        if step._sync_in_step:
            opt._grad_sync = step.sync
        opt.step()
        opt._grad_sync = None
    if side is not None:
        side.active = False
        side.join()
    if mode != "full":  # the plan's side stream is joined by the optimizer: join it here
        from twotower_amd import _lib

        torch.cuda.current_stream().wait_stream(_lib.side_stream(torch.device("cuda", 0)))
print("capture ended", flush=True)
g.replay()
torch.cuda.synchronize()
print(json.dumps({"mode": mode, "sync": sync, "xdev": xdev, "captured": True, "loss": float(loss)}), flush=True)
dist.destroy_process_group()
