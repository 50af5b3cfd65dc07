"""Data-parallel step on the real HIP kernels: two ranks share cuda:0 over gloo (RCCL will not
put two ranks on one GPU; the round-end 8-GPU run uses RCCL with the same code), and their
parameters after each step must equal a single process stepping on the global batch.

The DP step: each rank pools/scores its half, the in-batch candidates are all-gathered with
rank-offset labels, the loss is pre-scaled by 1/world, tower gradients are all-reduced, and the
table is updated from the all-gathered factored gradient on every rank ("gather"), by
reduce-scatter into row shards, AdamW per shard and all-gather ("shard"), or from the all-gathered
factored gradient on each row's owner only, then all-gather ("owner").  Sum orders differ from the single process (two partial sums), so the bar is the
fp32 1e-5 relative tolerance on the parameter change.  AdamW normalises every element's update,
which turns rounding-level differences of near-cancelled gradients (|g| ~ eps) into O(lr)
parameter differences; with eps = 1 and no decay the first update is -lr g / (|g| + 1), so the
parameter change measures the synchronised gradient itself, checked against the float64 oracle."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

WORLD = 2
LR = 1e6  # the parameter change dominates the O(1) parameters, so it is read back at fp32 precision
V, B, L = 3001, 64, 24
# tower widths E = H: 64 runs the library head (ops.TowerFF, outside ops.HEAD_WIDTHS); 128 and 256
# run the shipping hand-written head (tt_head_gemm, tt_head_wgrad2 on the "wgrad" side stream and
# the SideGrads join that the tower-gradient all-reduce waits on), with the in-batch operand prep
# in the head's normalise pass and the fused F.normalize backward where those shapes take them
WIDTHS = (64, 128, 256)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _build(loss_name, world, table_sync="auto", groups=False, E=64):
    import twotower_amd as tt

    torch.manual_seed(7)
    emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
    model = tt.build_two_tower("mean", emb, hidden_dim=E, tied_weights=True).to("cuda:0")
    if loss_name.startswith("in_batch"):
        kw = {"temperature": 0.1, "cross_device_negatives": world > 1,
              "compute_dtype": "bf16" if loss_name.endswith("bf16") else "fp32"}
    else:
        kw = {"margin": 0.2}
    params = model.parameters()
    if groups:  # e.g. no weight decay on biases: the gradient all-reduce must still run once per step
        named = dict(model.named_parameters())
        params = [{"params": [p for n, p in named.items() if not n.endswith("bias")]},
                  {"params": [p for n, p in named.items() if n.endswith("bias")], "weight_decay": 0.0}]
    opt = tt.optim.AdamW(params, lr=LR, eps=1.0, weight_decay=0.0, fused_tables=True, tables=[emb],
                         capturable=True, table_sync=table_sync)
    name = "in_batch" if loss_name.startswith("in_batch") else loss_name
    return model, tt.TrainStep(model, tt.losses.build(name, **kw), opt)


def _batch():
    import twotower_amd as tt

    return tt.data.synthetic_triplets(WORLD * B, L, V, seed=3, device="cuda:0")


def _worker(rank, port, loss_name, table_sync, q, inbatch_dp="owner", overlap="1", groups=False, E=64):
    # every process recomputes G in the backward (the default; the candidate-owner passes always
    # do), so single process and ranks form the same bf16 products
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TT_INBATCH_DP=inbatch_dp,
                      TT_INBATCH_BWD="recompute", TT_INBATCH_OVERLAP=overlap)
    try:
        torch.cuda.set_device(0)
        if rank >= 0:
            dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        from twotower_amd import _lib

        model, step = _build(loss_name, WORLD if rank >= 0 else 1, table_sync, groups, E)
        init = {n: p.detach().cpu().numpy().copy() for n, p in model.named_parameters()}
        full = _batch()
        b = full if rank < 0 else tuple(t[rank * B:(rank + 1) * B] for t in full)
        with _lib.record_calls() as calls:
            loss = step(*b).clone()
        torch.cuda.synchronize()
        if rank >= 0:
            dist.all_reduce(loss)
            loss /= WORLD
        # numpy arrays travel by value (torch CPU tensors would travel as fds of a dying process);
        # the parameters through state_dict(), which materialises a column-sharded table (every rank)
        sd = model.state_dict()
        delta = {n: sd[n].detach().cpu().numpy() - init[n] for n, _ in model.named_parameters()}
        q.put((rank, float(loss), init, delta, [t.cpu().numpy() for t in full], sorted(calls)))
    except Exception as e:
        import traceback

        q.put((rank, f"{e!r}\n{traceback.format_exc()}", None, None, None, None))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


KEYS = {"table": "query_tower.embedding.embedding.weight", "W1": "query_tower.feed_forward.0.weight",
        "b1": "query_tower.feed_forward.0.bias", "W2": "query_tower.feed_forward.2.weight",
        "b2": "query_tower.feed_forward.2.bias"}


def _check_head(E, calls, who):
    """The hand-written head ran at the widths it ships for (and its weight gradients as the
    one-launch pair on the side stream), the library head below them."""
    hand = {"tt_head_gemm", "tt_head_wgrad2"}
    if E in (128, 256):
        assert hand <= set(calls), (who, E, calls)
    else:
        assert not hand & set(calls), (who, E, calls)


def _run(loss_name, table_sync, inbatch_dp="owner", overlap="1", groups=False, E=64):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ref = ctx.Process(target=_worker, args=(-1, 0, loss_name, table_sync, q, "owner", "1", groups, E))
    ref.start()
    single = q.get(timeout=300)
    ref.join(timeout=60)
    assert single[2] is not None, single[1]
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, loss_name, table_sync, q, inbatch_dp, overlap, groups, E))
             for r in range(WORLD)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for r, loss, _, delta, _, _ in out:
        assert delta is not None, loss
    for who, calls in [("single", single[5])] + [(f"rank{o[0]}", o[5]) for o in out]:
        _check_head(E, calls, who)
    return single, out


_DP_CASES = [("in_batch", "gather", False), ("in_batch", "shard", False), ("triplet", "gather", False),
             ("triplet", "shard", False), ("triplet", "gather", True), ("in_batch", "shard", True),
             ("in_batch", "owner", False), ("triplet", "owner", True), ("in_batch", "column", False),
             ("triplet", "column", True)]


@pytest.mark.parametrize("E", WIDTHS)
@pytest.mark.parametrize("loss_name,table_sync,groups", _DP_CASES)
def test_dp_step_equals_global_batch(loss_name, table_sync, groups, E):
    """One step, eps 1, no decay: delta = -lr g / (|g| + 1), so g is recovered from the parameter
    change and compared with the float64 oracle on the global batch.  groups: the parameters in
    two param groups (weights with the table, biases apart), where a per-group all-reduce would
    sum the gradients twice.  E = H in WIDTHS: 128 and 256 are the shipping
    hand-written head (checked by the C-ABI calls each process made)."""
    from oracle import reference_math as O

    (_, r_loss, init, r_delta, ids, _), out = _run(loss_name, table_sync, groups=groups, E=E)
    params = {k: init[v] for k, v in KEYS.items()}
    kw = {"temperature": 0.1} if loss_name == "in_batch" else {"margin": 0.2}
    o_loss, _, o_grads = O.tied_step_grads(params, *ids, loss=loss_name, **kw)
    assert abs(r_loss - o_loss) < 1e-5
    runs = [("single", r_loss, r_delta)] + [(f"rank{r}", l_, d_) for r, l_, _, d_, _, _ in out]
    for name, loss, delta in runs:
        assert abs(loss - o_loss) < 1e-5, (name, loss, o_loss)
        for k, key in KEYS.items():
            d = delta[key].astype("float64")
            u = -d / LR
            g = u / (1.0 - abs(u))
            err = abs(g - o_grads[k]).max() / abs(o_grads[k]).max()
            assert err < 1e-5, (name, E, k, float(err))


@pytest.mark.parametrize("E", WIDTHS)
@pytest.mark.parametrize("inbatch_dp,overlap,table_sync", [("owner", "1", "gather"), ("owner", "0", "gather"),
                                                           ("allgather", "1", "gather"), ("owner", "1", "column")])
def test_dp_step_bf16_in_batch_equals_global_batch(inbatch_dp, overlap, table_sync, E):
    """bf16 scorer with cross-device negatives: candidate-owner gradients (bf16 copies gathered,
    no gradient reduce-scatter; the forward in two launches, own candidates scored while the
    others arrive, or in one launch after the gather) and the fp32-row all-gather + reduce-scatter
    form all give the single process's bf16 gradients on the global batch (same bf16 products,
    other fp32 sum orders), recovered from the parameter change as above."""
    (_, r_loss, _, r_delta, _, _), out = _run("in_batch_bf16", table_sync, inbatch_dp, overlap, E=E)

    def grads(delta):
        out = {}
        for k, key in KEYS.items():
            u = -delta[key].astype("float64") / LR
            out[k] = u / (1.0 - abs(u))
        return out

    want = grads(r_delta)
    for r, loss, _, delta, _, _ in out:
        assert abs(loss - r_loss) < 1e-5, (r, loss, r_loss)
        got = grads(delta)
        for k in KEYS:
            err = abs(got[k] - want[k]).max() / abs(want[k]).max()
            assert err < 1e-5, (inbatch_dp, E, r, k, float(err))


def _seed_worker(rank, port, q, seeds, Bq, M, H):
    import numpy as np

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        from twotower_amd import ops

        rng = np.random.default_rng(11)
        qa, da = rng.standard_normal((WORLD * Bq, H)), rng.standard_normal((WORLD * M, H))
        qa = torch.as_tensor(qa / np.linalg.norm(qa, axis=1, keepdims=True), dtype=torch.float32).bfloat16().float()
        da = torch.as_tensor(da / np.linalg.norm(da, axis=1, keepdims=True), dtype=torch.float32).bfloat16().float()
        Q = qa[rank * Bq:(rank + 1) * Bq].to("cuda:0").requires_grad_(True)
        D = da[rank * M:(rank + 1) * M].to("cuda:0").requires_grad_(True)
        loss = ops.InBatchSoftmaxLossOwned.apply(Q, D, 10.0, "bf16", None, None)
        loss.backward(torch.tensor(seeds[rank], device="cuda:0"))
        torch.cuda.synchronize()
        q.put((rank, Q.grad.cpu().numpy(), D.grad.cpu().numpy(), qa.numpy(), da.numpy()))
    except Exception as e:
        import traceback

        q.put((rank, f"{e!r}\n{traceback.format_exc()}", None, None, None))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("H", WIDTHS)
@pytest.mark.parametrize("seeds", [(0.5, 0.5), (0.3, 1.7), (0.0, 1.0)])
def test_owner_backward_takes_each_ranks_seed(seeds, H):
    """Candidate-owner gradients when the ranks seed their loss backward differently (ADVICE
    round 1): the objective is sum_r seed_r * loss_r, and the gradient of each rank's candidates
    must weigh every remote query's terms by that query's own rank seed.  Checked against float64
    autograd on the bf16-rounded operands at the bf16 scorer's bar."""
    import numpy as np

    Bq, M = 96, 192
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_seed_worker, args=(r, port, q, seeds, Bq, M, H)) for r in range(WORLD)]
    for p in procs:
        p.start()
    out = sorted((q.get(timeout=300) for _ in procs), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
    for r, dq, dd, qa, da in out:
        assert dd is not None, dq
    qa, da = (torch.as_tensor(out[0][3], dtype=torch.float64).requires_grad_(True),
              torch.as_tensor(out[0][4], dtype=torch.float64).requires_grad_(True))
    logits = qa @ da.T * 10.0
    labels = torch.cat([torch.arange(Bq) + r * M for r in range(WORLD)])
    ce = torch.nn.functional.cross_entropy(logits, labels, reduction="none")
    w = torch.cat([torch.full((Bq,), float(seeds[r]) / Bq, dtype=torch.float64) for r in range(WORLD)])
    (ce * w).sum().backward()
    for r, dq, dd, _, _ in out:
        for got, want in ((dq, qa.grad[r * Bq:(r + 1) * Bq]), (dd, da.grad[r * M:(r + 1) * M])):
            want = want.numpy()
            err = np.abs(got.astype(np.float64) - want).max() / max(np.abs(want).max(), 1e-30)
            assert err < 2e-3, (seeds, r, float(err))


@pytest.mark.gpu
@pytest.mark.parametrize("table_sync,loss_name", [("gather", "in_batch"), ("shard", "in_batch"),
                                                  ("shard", "multiple_negatives"), ("owner", "multiple_negatives"),
                                                  ("column", "in_batch"), ("column", "multiple_negatives")])
def test_dp_graph_replay_equals_eager_one_rank_rccl(table_sync, loss_name):
    """The N-rank step captured in one HIP graph (its RCCL collectives included: candidate
    all-gathers, the table exchange, the gradient all-reduce on the communication stream) replays
    exactly what the eager N-rank step computes: one RCCL rank with every exchange forced on
    (tests/_dp_graph_check.py, own process), five steps, losses and parameters bit for bit."""
    import json
    import subprocess
    import sys

    env = dict(os.environ, MASTER_PORT=str(_free_port()))
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "_dp_graph_check.py"), table_sync, loss_name], env=env,
                       capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["graph_kept"], res
    assert res["eager"] == res["graph"], res
    assert res["max_param_diff"] == 0.0, res


def _owner_vs_gather_worker(rank, port, q, Vt, steps):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        import twotower_amd as tt

        res = {}
        for mode in ("gather", "owner"):
            torch.manual_seed(5)
            emb = tt.embeddings.build("lookup", vocab_size=Vt, embedding_dim=128)
            model = tt.build_two_tower("mean", emb, hidden_dim=128, tied_weights=True).to("cuda:0")
            opt = tt.optim.AdamW(model.parameters(), lr=1e-2, fused_tables=True, tables=[emb], capturable=True,
                                 table_sync=mode)
            step = tt.TrainStep(model, tt.losses.build("triplet", margin=0.2), opt)
            for s in range(steps):
                full = tt.data.synthetic_triplets(WORLD * B, L, Vt, seed=20 + s, device="cuda:0")
                step(*(t[rank * B:(rank + 1) * B] for t in full))
            torch.cuda.synchronize()
            w = emb.embedding.weight
            sh = opt._shards.get(id(w))
            pad = None
            if sh is not None:  # the storage rows past V (the last chunks' padding) must stay zero
                pad = float(sh.storage()[sh.V:].abs().max()) if sh.Vp > sh.V else 0.0
                res["layout"] = (sh.NC, sh.R, sh.Vp)
            res[mode] = (w.detach().cpu().numpy().copy(), pad)
        q.put((rank, res))
    except Exception as e:
        import traceback

        q.put((rank, f"{e!r}\n{traceback.format_exc()}"))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("Vt", [17, 3001])
def test_owner_equals_gather_when_rows_do_not_divide(Vt):
    """the "owner" exchange at a vocabulary that is not a multiple of chunks x ranks.
    V = 3001 (NC 8, R 188): the last owned slab of rank 1 is clipped; V = 17 (NC 8, R 2): whole
    chunks are padding and some ranks own no row of a chunk at all, while the chunk is still
    all-gathered.  After two steps the table equals the replicated "gather" update bit for bit on
    every rank, and the padding rows of the storage stay zero."""
    import numpy as np

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_owner_vs_gather_worker, args=(r, port, q, Vt, 2)) for r in range(WORLD)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for r, res in out:
        assert isinstance(res, dict), res
        g, _ = res["gather"]
        o, pad = res["owner"]
        assert pad == 0.0, (r, pad, res["layout"])
        assert np.array_equal(g, o), (r, float(np.abs(g - o).max()), res["layout"])
    assert np.array_equal(out[0][1]["owner"][0], out[1][1]["owner"][0])
