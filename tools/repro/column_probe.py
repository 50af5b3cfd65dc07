"""One RCCL rank with every data-parallel exchange forced on (TT_DIST_FORCE=1) and the column-sharded
table (table_sync "column"): eager steps, then TrainStep's graph capture and replays, a line per
phase (flushed), so a hang names its phase.  Usage: python tools/repro/column_probe.py [in_batch|mn] [graph]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["TT_DIST_FORCE"] = "1"
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import twotower_amd as tt  # noqa: E402

t0 = time.time()


def say(msg):
    print(f"[{time.time() - t0:7.2f}s] {msg}", flush=True)


loss_name = sys.argv[1] if len(sys.argv) > 1 else "in_batch"
graph = len(sys.argv) > 2 and sys.argv[2] == "graph"
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
say("group up")
V, E, L, B, K = 3000, 256, 16, 256, 4
torch.manual_seed(0)
emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
model = tt.build_two_tower("mean", emb, hidden_dim=E, tied_weights=True).cuda()
if loss_name == "in_batch":
    loss_fn = tt.losses.build("in_batch", temperature=0.1, compute_dtype="bf16", cross_device_negatives=True)
else:
    mn = tt.losses.build("multiple_negatives", temperature=0.1)

    def loss_fn(q, p, n):
        return mn(q, p, n.view(q.shape[0], K, q.shape[1]))
opt = tt.optim.AdamW(model.parameters(), lr=1e-3, fused_tables=True, tables=[emb], capturable=True,
                     table_sync="column")
say(f"mode column: {hasattr(emb.embedding.weight, '_tt_column')}")
step = tt.TrainStep(model, loss_fn, opt, graph=graph, eager_steps=1)
negs = K if loss_name != "in_batch" else 1
batches = [tt.data.synthetic_triplets(B, L, V, seed=s, device="cuda", negatives=negs) for s in range(4)]
for s in range(4):
    say(f"step {s} issue")
    loss = step(*batches[s])
    torch.cuda.synchronize()
    say(f"step {s} done loss {float(loss):.6f} graph {step.graph}")
sd = model.state_dict()
say(f"state_dict ok, table sum {float(sd['query_tower.embedding.embedding.weight'].sum()):.6f}")
if len(sys.argv) > 3 and sys.argv[3] == "release":
    step.release()
    say("graphs released")
dist.barrier()
say("barrier ok")
dist.destroy_process_group()
say("done")
