"""Which RCCL collective forms survive HIP graph capture on this image?  One nccl rank (world 1,
127.0.0.1), one form per process, each captured then replayed twice and checked:

  sync_ar     dist.all_reduce on the current (capturing) stream, async_op=False
  async_ar    dist.all_reduce(async_op=True) + work.wait()
  side_ar     all_reduce issued on a side stream forked from / joined back to the capture stream
  gather      dist.all_gather_into_tensor on the current stream
  side_async_ar  async all-reduce + wait on a forked comm stream, joined by an event
  multi       all-gather on the capture stream, then a comm-stream async all-reduce
  unjoined    a side stream forked from the capture and never joined (no collective)
  step_gather the bench's DP TrainStep (--dp gather) captured through TrainStep(graph=True)

Usage: python tools/repro/capture_probe.py MODE   (prints one JSON line; segfaults are the finding)"""
import faulthandler
import json
import os
import sys

faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

mode = sys.argv[1]
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
torch.cuda.set_device(0)
x = torch.arange(1 << 16, device="cuda", dtype=torch.float32)
out = torch.empty_like(x)
warm = x.clone()
dist.all_reduce(warm)  # communicator set up outside the capture
torch.cuda.synchronize()


def body():
    if mode == "sync_ar":
        out.copy_(x)
        dist.all_reduce(out)
    elif mode == "async_ar":
        out.copy_(x)
        dist.all_reduce(out, async_op=True).wait()
    elif mode == "side_ar":
        s = side
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            out.copy_(x)
            dist.all_reduce(out)
        torch.cuda.current_stream().wait_stream(s)
    elif mode == "side_async_ar":  # GradSync.launch's pattern: async all-reduce on a comm stream
        side.wait_stream(torch.cuda.current_stream())
        out.copy_(x)
        with torch.cuda.stream(side):
            dist.all_reduce(out, async_op=True).wait()
            ev = torch.cuda.Event()
            ev.record(side)
        out.record_stream(side)
        torch.cuda.current_stream().wait_event(ev)
    elif mode == "multi":  # all-gather on the capture stream, then the comm-stream all-reduce
        tmp = torch.empty_like(x)
        dist.all_gather_into_tensor(tmp, x)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            out.copy_(tmp)
            dist.all_reduce(out, async_op=True).wait()
        torch.cuda.current_stream().wait_stream(side)
    elif mode == "unjoined":  # a forked stream never joined back: an error, or a crash?
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            out.copy_(x)
    elif mode == "gather":
        dist.all_gather_into_tensor(out, x)
    else:
        raise SystemExit(f"unknown mode {mode}")


res = {"mode": mode}
if mode == "step_gather":
    import twotower_amd as tt

    os.environ["TT_DIST_FORCE"] = "1"
    torch.manual_seed(0)
    emb = tt.embeddings.build("lookup", vocab_size=5000, embedding_dim=128)
    model = tt.build_two_tower("mean", emb, hidden_dim=128, tied_weights=True).cuda()
    loss = tt.losses.build("in_batch", temperature=0.1, compute_dtype="fp32", cross_device_negatives=True)
    opt = tt.optim.AdamW(model.parameters(), fused_tables=True, tables=[emb], capturable=True, table_sync="gather")
    step = tt.TrainStep(model, loss, opt, graph=True, eager_steps=1)
    batch = tt.data.synthetic_triplets(256, 16, 5000, seed=1, device="cuda")
    vals = [float(step(*batch)) for _ in range(3)]
    res.update(graph=step.graph, losses=vals)
else:
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g):
            body()
    except RuntimeError as e:
        res["error"] = str(e)[:300]
        print(json.dumps(res), flush=True)
        raise SystemExit(0)
    res["captured"] = True
    for _ in range(2):
        out.zero_()
        g.replay()
    torch.cuda.synchronize()
    res["ok"] = bool(torch.equal(out, x))
print(json.dumps(res), flush=True)
dist.destroy_process_group()
