"""Pre-flight for bench.py's N-rank HIP-graph step: every rank of the job runs this as a CHILD
process (its own RCCL world on MASTER_PORT, set by the parent to a free offset of the job's port),
which captures and replays a small N-rank TrainStep through the same code paths as the bench step
(cross-device in-batch loss or multiple-negatives, the chosen table exchange, the gradient
all-reduce).  The parent uses the graph only if every rank's child printed "canary ok", so a
capture that fails -- or crashes the process -- on this ROCm/RCCL stack costs the parent nothing
but the eager step.  Usage (by bench.py): python tools/dp_capture_canary.py --d 256 --loss in_batch
--negatives 1 --dtype bf16 --table-sync auto"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import twotower_amd as tt  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--loss", default="in_batch")
    ap.add_argument("--negatives", type=int, default=1)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--table-sync", default="auto")
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("nccl", rank=int(os.environ.get("RANK", "0")), world_size=world, device_id=dev)
    V, L, B, K = 4096, 16, 256, a.negatives
    torch.manual_seed(0)
    emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=a.d)
    model = tt.build_two_tower("mean", emb, hidden_dim=a.d, tied_weights=True).to(dev)
    if a.loss == "in_batch":
        loss_fn = tt.losses.build("in_batch", temperature=0.1, compute_dtype=a.dtype, cross_device_negatives=True)
    else:
        mn = tt.losses.build("multiple_negatives", temperature=0.1)

        def loss_fn(q, p, n):
            return mn(q, p, n.view(q.shape[0], K, q.shape[1]))
    opt = tt.optim.AdamW(model.parameters(), lr=1e-3, fused_tables=True, tables=[emb], capturable=True,
                         table_sync=a.table_sync)
    step = tt.TrainStep(model, loss_fn, opt, graph=True, eager_steps=1)
    batch = tt.data.synthetic_triplets(B, L, V, seed=dist.get_rank(), device=dev,
                                       negatives=max(K, 1))[:(2 if K == 0 else 3)]
    losses = [float(step(*batch)) for _ in range(3)]
    torch.cuda.synchronize()
    graphed = step.graph
    step.release()  # before the process group goes: a captured all-to-all holds RCCL resources
    dist.barrier()
    dist.destroy_process_group()
    if graphed and all(math.isfinite(x) for x in losses):
        print(f"canary ok: losses {losses}", flush=True)
        return 0
    print(f"canary failed: graph {step.graph}, losses {losses}", flush=True)
    return 1


if __name__ == "__main__":
    sys.exit(main())
