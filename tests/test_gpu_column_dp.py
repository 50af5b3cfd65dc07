"""The column-sharded table exchange (table_sync "column", distributed.ColumnTable) end to end through
TrainStep on the real HIP kernels, ranks sharing cuda:0 over gloo:

  * world size 4 at E = H = 128, so each rank owns El = 32 columns -- the slab width of C5 at N = 8 --
    for the triplet, multiple-negatives and bf16 in-batch losses: the ids all-gather, the pooled and
    gs all-to-alls and the merged per-rank plans (tt_bag_col_reduce_ex) against the float64 oracle on
    the global batch (per-sample losses) or the single process on the global batch (bf16 in-batch);
  * a checkpoint round trip in column mode (twotower/utils.py:231-330): two steps, save_checkpoint
    (model + optim.AdamW state), fresh ranks load it and step once more -- bit for bit the
    uninterrupted third step, and the saved moments full width under torch's keys;
  * release_tables() after a column step, then a dense step (the moments must be gathered
    to V x E first);
  * evaluation without gradient: stale table -> the collective column forward; after state_dict()
    (which materialises the slabs) rank 0 alone runs a forward on its local weight, and both equal.

The recovered-gradient trick of test_gpu_dp.py: eps 1, no decay, lr 1e6, so one AdamW step is
-lr g / (|g| + 1) and g is read back from the parameter change."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

LR = 1e6
V, B, L, K = 3001, 32, 24, 2  # B queries per rank; K negatives per query (multiple negatives)
KEYS = {"table": "query_tower.embedding.embedding.weight", "W1": "query_tower.feed_forward.0.weight",
        "b1": "query_tower.feed_forward.0.bias", "W2": "query_tower.feed_forward.2.weight",
        "b2": "query_tower.feed_forward.2.bias"}


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _loss(name, dp):
    import twotower_amd as tt

    if name == "in_batch_bf16":
        return tt.losses.build("in_batch", temperature=0.1, compute_dtype="bf16", cross_device_negatives=dp)
    if name == "multiple_negatives":
        mn = tt.losses.build("multiple_negatives", temperature=0.1)

        def fn(q, p, n):
            return mn(q, p, n.view(q.shape[0], K, q.shape[1]))
        return fn
    return tt.losses.build("triplet", margin=0.2)


def _build(loss_name, dp, table_sync, E, lr=LR, eps=1.0, wd=0.0, seed=7):
    import twotower_amd as tt

    torch.manual_seed(seed)
    emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
    model = tt.build_two_tower("mean", emb, hidden_dim=E, tied_weights=True).to("cuda:0")
    opt = tt.optim.AdamW(model.parameters(), lr=lr, eps=eps, weight_decay=wd, fused_tables=True, tables=[emb],
                         capturable=True, table_sync=table_sync)
    return emb, model, opt, tt.TrainStep(model, _loss(loss_name, dp), opt)


def _batch(world, seed, negs):
    import twotower_amd as tt

    return tt.data.synthetic_triplets(world * B, L, V, seed=seed, device="cuda:0", negatives=negs)


def _shard(full, rank, negs):
    q, p, n = full
    return q[rank * B:(rank + 1) * B], p[rank * B:(rank + 1) * B], n[rank * B * negs:(rank + 1) * B * negs]


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TT_INBATCH_BWD="recompute")
    torch.cuda.set_device(0)
    if rank >= 0:
        dist.init_process_group("gloo", rank=rank, world_size=world)


def _spawn(target, world, *args, timeout=300):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=timeout) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    out.sort(key=lambda t: t[0])
    for o in out:
        assert not isinstance(o[1], str), o[1]
    return out


def _spawn_single(target, world, *args, timeout=300):
    """One process without a process group (rank -1) on the global batch of `world` ranks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=target, args=(-1, world, 0, q) + args)
    p.start()
    out = q.get(timeout=timeout)
    p.join(timeout=60)
    assert not isinstance(out[1], str), out[1]
    return out


# ------------------------------------------------------------------------------------------------
# world size 4, El = 32
def _w4_worker(rank, world, port, q, loss_name, E):
    try:
        _init(rank, world, port)
        from twotower_amd import _lib

        negs = K if loss_name == "multiple_negatives" else 1
        emb, model, opt, step = _build(loss_name, rank >= 0, "column" if rank >= 0 else "auto", E)
        init = {n: p.detach().cpu().numpy().copy() for n, p in model.named_parameters()}
        full = _batch(world, 3, negs)
        b = full if rank < 0 else _shard(full, rank, negs)
        with _lib.record_calls() as calls:
            loss = step(*b).clone()
        torch.cuda.synchronize()
        if rank >= 0:
            dist.all_reduce(loss)
            loss /= world
            col = opt._columns[id(emb.embedding.weight)]
            assert col.El == E // world
        sd = model.state_dict()  # materialises the column slabs (collective)
        delta = {n: sd[n].detach().cpu().numpy() - init[n] for n, _ in model.named_parameters()}
        q.put((rank, (float(loss), init, delta, [t.cpu().numpy() for t in full], sorted(calls))))
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, f"{e!r}\n{traceback.format_exc()}"))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _grads_from(delta):
    out = {}
    for k, key in KEYS.items():
        u = -delta[key].astype("float64") / LR
        out[k] = u / (1.0 - abs(u))
    return out


def _oracle_grads(loss_name, params, q, p, n):
    from oracle import reference_math as O

    if loss_name == "triplet":
        loss, _, g = O.tied_step_grads(params, q, p, n, loss="triplet", margin=0.2)
        return loss, g
    qo, qc = O.tower_fwd(params, q)
    po, pc = O.tower_fwd(params, p)
    no, nc = O.tower_fwd(params, n)
    loss, (dq, dp, dn) = O.multi_neg_fwd_bwd(qo, po, no.reshape(qo.shape[0], K, -1), 0.1)
    g = None
    for dout, cache in ((dq, qc), (dp, pc), (dn.reshape(no.shape), nc)):
        gi = O.tower_bwd(params, dout, cache)
        g = gi if g is None else {k: g[k] + gi[k] for k in g}
    return loss, g


@pytest.mark.parametrize("loss_name", ["triplet", "multiple_negatives", "in_batch_bf16"])
def test_column_world4_el32_equals_global_batch(loss_name):
    world, E = 4, 128
    out = _spawn(_w4_worker, world, loss_name, E)
    for r, (_, _, _, _, calls) in out:
        assert "tt_bag_col_reduce_ex" in calls and "tt_bag_mean_fwd_cols" in calls, (r, calls)
        assert "tt_head_gemm" in calls, (r, calls)  # the shipping hand-written head at H = 128
    if loss_name == "in_batch_bf16":  # the single process on the global batch forms the same bf16 products
        single = _spawn_single(_w4_worker, world, loss_name, E)
        r_loss, _, r_delta, _, _ = single[1]
        want = _grads_from(r_delta)
        for r, (loss, _, delta, _, _) in out:
            assert abs(loss - r_loss) < 1e-5, (r, loss, r_loss)
            got = _grads_from(delta)
            for k in KEYS:
                err = abs(got[k] - want[k]).max() / abs(want[k]).max()
                assert err < 1e-5, (r, k, float(err))
        return
    loss0, init, _, ids, _ = out[0][1]
    params = {k: init[v] for k, v in KEYS.items()}
    o_loss, o_grads = _oracle_grads(loss_name, params, *ids)
    for r, (loss, _, delta, _, _) in out:
        assert abs(loss - o_loss) < 1e-5, (r, loss, o_loss)
        got = _grads_from(delta)
        for k in KEYS:
            err = abs(got[k] - o_grads[k]).max() / abs(o_grads[k]).max()
            assert err < 1e-5, (r, k, float(err))


# ------------------------------------------------------------------------------------------------
# checkpoint round trip, column mode
def _ckpt_worker(rank, world, port, q, phase, path):
    try:
        _init(rank, world, port)
        from twotower_amd import checkpoint

        E = 128
        emb, model, opt, step = _build("in_batch_bf16", True, "column", E, lr=1e-2, eps=1e-8, wd=0.01,
                                       seed=7 if phase != "resume" else 99)
        batches = [_shard(_batch(world, 40 + s, 1), rank, 1) for s in range(3)]
        res = {}
        if phase == "full":
            for s in range(3):
                step(*batches[s])
        elif phase == "save":
            for s in range(2):
                step(*batches[s])
            checkpoint.save_checkpoint(model, {"a": 1}, opt, epoch=1, loss=0.5, checkpoint_dir=os.path.dirname(path),
                                       checkpoint_name=os.path.basename(path), save_best=False)
            dist.barrier()
        else:  # resume: fresh model / optimizer (other init), the checkpoint, the third step
            checkpoint.load_checkpoint(path, model, opt, device="cuda:0")
            step(*batches[2])
        torch.cuda.synchronize()
        sd = model.state_dict()
        res["params"] = {k: v.detach().cpu().numpy().copy() for k, v in sd.items()}
        osd = opt.state_dict()
        w = emb.embedding.weight
        idx = [i for i, p in enumerate(p for g in opt.param_groups for p in g["params"]) if p is w][0]
        res["moment_shape"] = tuple(osd["state"][idx]["exp_avg"].shape)
        res["moment_v"] = osd["state"][idx]["exp_avg_sq"].detach().cpu().numpy().copy()
        q.put((rank, res))
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, f"{e!r}\n{traceback.format_exc()}"))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_column_checkpoint_round_trip_bit_equal():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "col.pt")
        full = _spawn(_ckpt_worker, world, "full", path)
        _spawn(_ckpt_worker, world, "save", path)
        saved = torch.load(path, map_location="cpu", weights_only=True)
        resumed = _spawn(_ckpt_worker, world, "resume", path)
    st = saved["optimizer"]["state"]
    table_states = [s for s in st.values() if s["exp_avg"].dim() == 2 and s["exp_avg"].shape[0] == V]
    assert table_states and all(tuple(s["exp_avg"].shape) == (V, 128) for s in table_states)  # full width
    assert all(set(s) >= {"step", "exp_avg", "exp_avg_sq"} for s in st.values())
    assert tuple(saved["model"][KEYS["table"]].shape) == (V, 128)
    for (r, a), (_, b) in zip(full, resumed):
        assert a["moment_shape"] == (V, 128)
        for k in a["params"]:
            assert np.array_equal(a["params"][k], b["params"][k]), (r, k, float(np.abs(a["params"][k] -
                                                                                     b["params"][k]).max()))
        assert np.array_equal(a["moment_v"], b["moment_v"]), r


# ------------------------------------------------------------------------------------------------
# release_tables() after column / shard steps, then a dense step
def _release_worker(rank, world, port, q, mode):
    try:
        _init(rank, world, port)
        E = 128
        emb, model, opt, step = _build("triplet", True, mode, E, lr=1e-2, eps=1e-8, wd=0.01)
        step(*_shard(_batch(world, 50, 1), rank, 1))
        opt.release_tables()
        w = emb.embedding.weight
        st = opt.state[w]
        shapes = (tuple(st["exp_avg"].shape), tuple(st["exp_avg_sq"].shape))
        # a plain dense step on the same global batch on every rank (no exchange: identical grads)
        qf, pf, nf = _batch(world, 51, 1)
        opt.zero_grad()
        lf = _loss("triplet", False)
        loss = lf(*model(qf, pf, nf))
        loss.backward()
        opt.step()
        torch.cuda.synchronize()
        q.put((rank, {"shapes": shapes, "table": w.detach().cpu().numpy().copy(),
                      "m": st["exp_avg"].detach().cpu().numpy().copy()}))
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, f"{e!r}\n{traceback.format_exc()}"))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_release_tables_then_dense_step():
    world = 2
    res = {mode: _spawn(_release_worker, world, mode) for mode in ("column", "shard", "gather")}
    ref = res["gather"][0][1]
    for mode in ("column", "shard"):
        for r, out in res[mode]:
            assert out["shapes"] == ((V, 128), (V, 128)), (mode, r, out["shapes"])
            err = np.abs(out["table"] - ref["table"]).max() / np.abs(ref["table"]).max()
            assert err < 1e-5, (mode, r, float(err))
            merr = np.abs(out["m"] - ref["m"]).max() / np.abs(ref["m"]).max()
            assert merr < 1e-5, (mode, r, float(merr))
        assert np.array_equal(res[mode][0][1]["table"], res[mode][1][1]["table"]), mode


# ------------------------------------------------------------------------------------------------
# evaluation without gradient on a column table
def _eval_worker(rank, world, port, q):
    try:
        _init(rank, world, port)
        from twotower_amd import _lib

        emb, model, opt, step = _build("triplet", True, "column", 128, lr=1e-2, eps=1e-8, wd=0.01)
        step(*_shard(_batch(world, 60, 1), rank, 1))
        col = opt._columns[id(emb.embedding.weight)]
        qids = _batch(world, 61, 1)[0][:B]  # the same query ids on every rank
        with torch.no_grad():
            assert col.stale
            with _lib.record_calls() as c1:
                a = model.query_tower(qids).clone()  # stale: the collective column forward (all ranks)
        model.state_dict()  # materialises (collective)
        res = {"stale_calls": sorted(c1)}
        if rank == 0:  # rank 0 alone: a rank-local forward on the materialised weight
            with torch.no_grad(), _lib.record_calls() as c2:
                b = model.query_tower(qids)
            torch.cuda.synchronize()
            res["equal"] = bool(torch.equal(a, b))
            res["local_calls"] = sorted(c2)
        q.put((rank, res))
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, f"{e!r}\n{traceback.format_exc()}"))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_column_no_grad_forward_rank_local_after_materialize():
    out = _spawn(_eval_worker, 2, timeout=240)
    r0 = out[0][1]
    assert "tt_bag_mean_fwd_cols" in r0["stale_calls"]
    assert r0["equal"]
    assert "tt_bag_mean_fwd_cols" not in r0["local_calls"]
    assert any(c.startswith("tt_bag_mean_fwd") for c in r0["local_calls"]), r0["local_calls"]
