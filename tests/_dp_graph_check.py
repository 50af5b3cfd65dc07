"""Run by test_gpu_dp.py::test_dp_graph_replay_equals_eager_one_rank_rccl in its own process:
one RCCL rank with every data-parallel exchange forced on (TT_DIST_FORCE=1), two identical
models, one stepped eagerly and one by TrainStep's captured graph, on the same batches; prints
one JSON line with the largest parameter difference and both loss lists (they must be equal bit
for bit: the replay issues the same kernels and collectives in the same order)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["TT_DIST_FORCE"] = "1"
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import twotower_amd as tt  # noqa: E402

table_sync, loss_name = sys.argv[1], sys.argv[2]
modes = (False, True) if len(sys.argv) < 4 else tuple(m == "graph" for m in sys.argv[3].split(","))
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
V, E, L, B, K = 3000, 256, 16, 256, 4


def build(graph):
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
                         table_sync=table_sync)
    return model, tt.TrainStep(model, loss_fn, opt, graph=graph, eager_steps=1)


negs = K if loss_name != "in_batch" else 1
batches = [tt.data.synthetic_triplets(B, L, V, seed=s, device="cuda", negatives=negs) for s in range(4)]
out = []
for graph in modes:
    model, step = build(graph)
    losses = [float(step(*batches[s % 4])) for s in range(5)]
    torch.cuda.synchronize()
    out.append((losses, {k: v.detach().clone() for k, v in model.state_dict().items()}, step.graph))
    step.release()  # before the process group goes: a captured all-to-all holds RCCL resources
diff = max(float((out[1][1][k] - out[0][1][k]).abs().max()) for k in out[1][1])
print(json.dumps({"eager": out[0][0], "graph": out[1][0], "max_param_diff": diff, "modes": sys.argv[3:],
                  "graph_kept": out[1][2] == modes[1]}), flush=True)
dist.destroy_process_group()
