"""Data-parallel logic on CPU: gloo, world_size 2, one process per rank (the same code runs over
RCCL on the GPU node).  Each check compares the 2-rank computation against the single-process
computation on the concatenated global batch, with torch CPU math standing in for the HIP
kernels (which need a GPU): the collectives, the row sharding, the label offsets and the loss
scaling are what is under test here."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F

from twotower_amd import distributed as D

WORLD = 2


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(fn, *args):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_entry, args=(r, port, fn, q, args)) for r in range(WORLD)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    errs = [r for r in results if isinstance(r, str)]
    assert not errs, errs[0]


def _entry(rank, port, fn, q, args):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        torch.manual_seed(0)
        fn(rank, *args)
        q.put(None)
    except Exception as e:  # reported to the parent
        import traceback

        q.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


# ---------------------------------------------------------------------------------------------
def _collectives(rank):
    x = torch.arange(6 * 3, dtype=torch.float32).view(6, 3) * (rank + 1)
    out = torch.empty(3, 3)
    D.reduce_scatter_rows(out, x)
    full = torch.arange(18, dtype=torch.float32).view(6, 3) * 3  # (1 + 2) x
    assert torch.equal(out, full[rank * 3:(rank + 1) * 3])
    g = torch.empty(4, 2)
    D.all_gather_rows(g, torch.full((2, 2), float(rank)))
    assert torch.equal(g, torch.tensor([[0., 0.], [0., 0.], [1., 1.], [1., 1.]]))
    # in place: the input is this rank's slab of the output
    buf = torch.zeros(4, 2)
    buf[rank * 2:(rank + 1) * 2] = rank + 5
    D.all_gather_rows(buf, buf[rank * 2:(rank + 1) * 2])
    assert torch.equal(buf, torch.tensor([[5., 5.], [5., 5.], [6., 6.], [6., 6.]]))


def test_collectives_gloo():
    _run(_collectives)


# ---------------------------------------------------------------------------------------------
def _ref_adamw(p, g, m, v, step, lr=1e-3, b1=0.9, b2=0.999, eps=1e-8, wd=0.01):
    p.mul_(1 - lr * wd)
    m.lerp_(g, 1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    denom = (v.sqrt() / (1 - b2 ** step) ** 0.5).add_(eps)
    p.addcdiv_(m, denom, value=-lr / (1 - b1 ** step))


def _sharded_table(rank, V, chunks):
    """Row-sharded AdamW on the reduce-scattered gradient == full AdamW on the global gradient,
    with the rows in `chunks` chunks of interleaved ownership (each chunk's slabs updated on
    their own, as optim.AdamW's pipelined exchange does); the sharded moments gather back into
    the full layout (state_dict) and split again (load)."""
    E = 4
    torch.manual_seed(1)
    table0 = torch.randn(V, E)
    grads = [torch.randn(V, E) for _ in range(WORLD)]  # each rank's local (pre-scaled) gradient
    w = torch.nn.Parameter(table0.clone())
    sh = D.ShardedRows(w, None, chunks=chunks)
    assert sh.NC == chunks and sh.Vp == chunks * WORLD * sh.R and sh.Vp >= V and w.shape == (V, E)
    m = torch.zeros(sh.Vs, E)
    v = torch.zeros(sh.Vs, E)
    ref_p, ref_m, ref_v = table0.clone(), torch.zeros(V, E), torch.zeros(V, E)
    for step in (1, 2, 3):
        gbuf = sh.new_grad_buffer()
        gbuf[:V] = grads[rank] * step
        g_shard = sh.reduce_scatter(gbuf)
        st = sh.storage()
        for c in range(sh.NC):
            _ref_adamw(sh.own(st, c), sh.shard_chunk(g_shard, c), sh.shard_chunk(m, c), sh.shard_chunk(v, c), step)
        sh.all_gather_params()
        _ref_adamw(ref_p, sum(g * step for g in grads), ref_m, ref_v, step)
        assert torch.allclose(w.data, ref_p, rtol=0, atol=1e-6), step
    if sh.Vp > V:
        assert torch.equal(sh.storage()[V:], torch.zeros(sh.Vp - V, E))  # padding rows stay zero
    full = sh.gather_full(m)
    assert torch.allclose(full[:V], ref_m, rtol=0, atol=1e-6)  # the full-layout moments (state_dict)
    assert torch.equal(sh.rows(full), m)                       # ... and back to this rank's rows (load)


@pytest.mark.parametrize("V,chunks", [(10, 1), (11, 1), (11, 3), (40, 4)])
def test_sharded_table_adamw_equals_global(V, chunks):
    _run(_sharded_table, V, chunks)


# ---------------------------------------------------------------------------------------------
def _inbatch_ref(q, d, tau, off):
    s = q @ d.t() / tau
    return F.cross_entropy(s, torch.arange(q.shape[0]) + off)


def _cross_device_negatives(rank):
    """Local loss on all-gathered candidates with offset labels, pre-scaled by 1/world and
    summed over ranks == the global-batch in-batch loss; gradients flow back to the owners."""
    B, H, tau = 5, 8, 0.1
    torch.manual_seed(2)
    qg = torch.randn(WORLD * B, H)
    dg = torch.randn(WORLD * 2 * B, H)  # each rank holds 2B candidates (its p and n)
    q = qg[rank * B:(rank + 1) * B].clone().requires_grad_(True)
    d = dg[rank * 2 * B:(rank + 1) * 2 * B].clone().requires_grad_(True)
    dall, off = D.gather_candidates(d)
    assert off == rank * 2 * B and dall.shape[0] == WORLD * 2 * B
    # labels: query i of rank r is positive for candidate row off + i (its own p)
    loss = _inbatch_ref(q, dall, tau, off)
    (loss / WORLD).backward()
    total = loss.detach().clone()
    dist.all_reduce(total)
    # global reference: the same candidates, labels = each query's own positive row
    qr = qg.clone().requires_grad_(True)
    dr = dg.clone().requires_grad_(True)
    labels = torch.cat([torch.arange(B) + r * 2 * B for r in range(WORLD)])
    ref = F.cross_entropy(qr @ dr.t() / tau, labels)
    ref.backward()
    assert torch.allclose(total / WORLD, ref.detach(), atol=1e-6)
    assert torch.allclose(q.grad, qr.grad[rank * B:(rank + 1) * B], atol=1e-6)
    assert torch.allclose(d.grad, dr.grad[rank * 2 * B:(rank + 1) * 2 * B], atol=1e-6)


def test_cross_device_negatives_equal_global_batch():
    _run(_cross_device_negatives)


def _grad_sync(rank):
    lin = torch.nn.Linear(3, 2)
    sync = D.GradSync(lin.parameters())
    assert sync.loss_scale() == 0.5
    x = torch.full((4, 3), float(rank + 1))
    (lin(x).sum() * sync.loss_scale()).backward()
    sync.sync()
    # mean over the two ranks' gradients
    assert torch.allclose(lin.weight.grad, torch.full((2, 3), 4 * 1.5))
    assert torch.allclose(lin.bias.grad, torch.full((2,), 4.0))


def test_grad_sync_mean():
    _run(_grad_sync)


def _sync_modes(rank):
    assert D.table_sync_mode("auto") == "gather"  # 2 ranks
    assert D.table_sync_mode("shard") == "shard"
    try:
        D.table_sync_mode("bogus")
    except ValueError:
        pass
    else:
        raise AssertionError("bad mode accepted")


def test_table_sync_mode_selection():
    assert D.table_sync_mode("auto") == "local"  # no process group
    _run(_sync_modes)


def test_child_world_env_under_torchrun():
    """bench.py's capture canary runs a child per rank that forms its own process group of the
    same ranks: under torch.distributed.run (agent store on the job's port) the children must get
    their own port and store (bench.child_world_env); 2 ranks, gloo, CPU."""
    import socket
    import subprocess
    import sys

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ)
    env.pop("TT_DIST_FORCE", None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port),
                        os.path.join(here, "_child_world_check.py")],
                       env=env, capture_output=True, text=True, timeout=240, cwd=os.path.dirname(here))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert r.stdout.count("child ok") == 2, r.stdout[-2000:] + r.stderr[-2000:]


# ---------------------------------------------------------------------------------------------
# Quantities that size collectives must agree across ranks (ShardedRows' chunk count).
def _agree_chunks(rank):
    assert D._agree(8, None, torch.device("cpu"), "x") == 8
    with pytest.raises(ValueError, match="disagree"):
        D._agree(8 if rank == 0 else 4, None, torch.device("cpu"), "row chunks")
    w = torch.nn.Parameter(torch.zeros(40, 4))
    os.environ["TT_SHARD_CHUNKS"] = "4" if rank == 0 else "2"
    with pytest.raises(ValueError, match="TT_SHARD_CHUNKS"):
        D.ShardedRows(w)
    os.environ["TT_SHARD_CHUNKS"] = "2"
    assert D.ShardedRows(w).NC == 2


def test_sharded_chunks_agree_across_ranks_gloo():
    _run(_agree_chunks)


# ---------------------------------------------------------------------------------------------
# The N-rank HIP-graph capture is refused (TrainStep stays eager) where ProcessGroupNCCL's event
# cache may be on: its watchdog aborts the process on a recycled event under capture (round 3).
def test_capture_blocker_rules(monkeypatch):
    monkeypatch.setattr(D.dist, "is_initialized", lambda: True)
    monkeypatch.setattr(D.dist, "get_backend", lambda group=None: "nccl")
    monkeypatch.setitem(D._AT_IMPORT, "group_existed", False)
    monkeypatch.setitem(D._AT_IMPORT, "event_cache", None)
    monkeypatch.setenv("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
    assert D.capture_blocker() is None  # group created after the import, the default applied
    monkeypatch.setenv("TORCH_NCCL_CUDA_EVENT_CACHE", "1")  # the caller turned the cache back on
    assert "TORCH_NCCL_CUDA_EVENT_CACHE" in D.capture_blocker()
    monkeypatch.setenv("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
    monkeypatch.setitem(D._AT_IMPORT, "group_existed", True)  # a group created before the import ...
    assert "before twotower_amd.distributed was imported" in D.capture_blocker()  # ... variable unset
    monkeypatch.setitem(D._AT_IMPORT, "event_cache", "1")  # ... with the cache on
    assert "before twotower_amd.distributed was imported" in D.capture_blocker()
    monkeypatch.setitem(D._AT_IMPORT, "event_cache", "0")  # ... with the cache off
    assert D.capture_blocker() is None
    monkeypatch.setattr(D.dist, "get_backend", lambda group=None: "cuda:nccl,cpu:gloo")  # mixed: nccl rules
    monkeypatch.setitem(D._AT_IMPORT, "event_cache", None)
    assert "before twotower_amd.distributed was imported" in D.capture_blocker()
    monkeypatch.setattr(D.dist, "get_backend", lambda group=None: "gloo")
    assert "gloo" in D.capture_blocker()


def test_capture_blocker_group_before_import_unset_variable():
    """a process group created before the module's import with the variable unset:
    the import-time record must keep 'unset' (not the default the import then applies), so the
    capture is refused."""
    import subprocess
    import sys

    code = """
import os, sys, torch.distributed as dist
sys.path.insert(0, %r)
os.environ.pop("TORCH_NCCL_CUDA_EVENT_CACHE", None)
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(%d))
dist.init_process_group("gloo", rank=0, world_size=1)
import twotower_amd.distributed as D
assert D._AT_IMPORT == {"event_cache": None, "group_existed": True}, D._AT_IMPORT
assert os.environ["TORCH_NCCL_CUDA_EVENT_CACHE"] == "0"
dist.get_backend = lambda group=None: "nccl"
why = D.capture_blocker()
assert why is not None and "before" in why, why
print("ok")
""" % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))), _free_port())
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]


def test_capture_error_classification():
    from twotower_amd.train_step import _is_capture_error

    assert _is_capture_error(RuntimeError("operation not permitted when stream is capturing"))
    assert _is_capture_error(RuntimeError("hipErrorStreamCaptureUnsupported"))
    assert not _is_capture_error(RuntimeError("mat1 and mat2 shapes cannot be multiplied"))
    # unrelated errors that merely contain the words a substring match used to take
    assert not _is_capture_error(RuntimeError("value not permitted for this argument"))
    assert not _is_capture_error(RuntimeError("the captured tensor was freed"))


def test_deferred_loss_mean_only_for_the_bare_in_batch_loss():
    """TrainStep lets the in-batch loss leave its mean to the backward only when loss_fn returns
    that loss itself (a wrapped loss read the unformed value)."""
    import twotower_amd as tt

    emb = tt.embeddings.build("lookup", vocab_size=50, embedding_dim=16)
    model = tt.build_two_tower("mean", emb, hidden_dim=16, tied_weights=True)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    bare = tt.losses.build("in_batch", temperature=0.1, compute_dtype="bf16")
    assert tt.TrainStep(model, bare, opt)._defer_mean
    assert tt.TrainStep(model, tt.losses.in_batch_sampled_softmax_loss, opt)._defer_mean
    assert not tt.TrainStep(model, lambda q, p, n: 0.5 * bare(q, p, n), opt)._defer_mean
    assert not tt.TrainStep(model, tt.losses.build("in_batch", cross_device_negatives=True), opt)._defer_mean
    assert not tt.TrainStep(model, tt.losses.build("triplet"), opt)._defer_mean


# ---------------------------------------------------------------------------------------------
# Column-sharded table (table_sync "column"): the exchanges of BagMeanPoolColumn around the HIP
# kernels, with torch CPU pooling / scatter standing in for tt_bag_mean_fwd / tt_bag_col_reduce.
def _column_flow(rank):
    from twotower_amd import ops

    V, E, nseq, L = 37, 64, 5, 7
    g = torch.Generator().manual_seed(3)
    table = torch.randn(V, E, generator=g)
    ids_all = torch.randint(0, V, (WORLD * nseq, L), generator=g)  # the global batch, rank-major
    dpool_all = torch.randn(WORLD * nseq, E, generator=g)
    w = torch.nn.Parameter(table.clone())
    col = D.ColumnTable(w, None)
    assert col.El == E // WORLD and torch.equal(col.slab, table[:, rank * col.El:(rank + 1) * col.El])

    def pool(t, ids):  # encoders.py:62-72 on CPU
        m = (ids > 0).float()
        return (t[ids] * m[..., None]).sum(1) / (m.sum(1, keepdim=True) + 1e-9)

    # all-to-all semantics
    x = torch.arange(WORLD * 3 * 2, dtype=torch.float32).view(WORLD * 3, 2) + 100 * rank
    y = torch.empty_like(x)
    D.all_to_all_rows(y, x)
    for s in range(WORLD):
        assert torch.equal(y[s * 3:(s + 1) * 3], torch.arange(rank * 3 * 2, (rank + 1) * 3 * 2,
                                                             dtype=torch.float32).view(3, 2) + 100 * s)
    # forward: this rank's columns for every rank's sequences -> this rank's whole pooled rows
    part = pool(col.slab, ids_all)
    pooled = ops.column_pooled_exchange(part, col, nseq)
    want = pool(table, ids_all[rank * nseq:(rank + 1) * nseq])
    assert torch.allclose(pooled, want, rtol=1e-6, atol=1e-6)
    # backward: this rank's gs -> every rank's gs at this rank's columns
    gs_all = ops.column_grad_exchange(dpool_all[rank * nseq:(rank + 1) * nseq].contiguous(), col)
    assert torch.equal(gs_all, dpool_all[:, col.c0:col.c0 + col.El])
    # slabs back into the parameter, moments to full width and back
    col.slab.mul_(2.0)
    col.stale = True
    col.materialize()
    assert torch.equal(w.data, table * 2.0) and not col.stale
    m = col.slab * 3.0
    full = col.gather_cols(m)
    assert torch.equal(full, table * 6.0) and torch.equal(col.own_cols(full), m)
    w.data.copy_(table)
    col.load_from_weight()
    assert torch.equal(col.slab, table[:, col.c0:col.c0 + col.El])


def test_column_table_exchanges_gloo():
    _run(_column_flow)


def test_column_mode_selection(monkeypatch):
    monkeypatch.setattr(D, "is_active", lambda group=None: True)
    monkeypatch.setattr(D.dist, "get_world_size", lambda group=None: 8)
    # "column" is opt-in (its forwards and state_dict() are collective); "auto" keeps a
    # replicated table: gather up to 4 ranks, shard beyond
    assert D.table_sync_mode("auto", None, E=256) == "shard"
    assert D.table_sync_mode("auto", None, E=48) == "shard"
    assert D.table_sync_mode("column", None, E=256) == "column"  # C3 / C4 / C5 at N = 8: 32 columns each
    monkeypatch.setattr(D.dist, "get_world_size", lambda group=None: 2)
    assert D.table_sync_mode("auto", None, E=256) == "gather"
    assert D.table_sync_mode("column", None, E=256) == "column"  # 128 columns each
    assert D.column_ok(256, 8) and D.column_ok(256, 2) and not D.column_ok(1024, 2)  # 512 columns: past the slabs
    assert not D.column_ok(256, 3) and D.column_ok(128, 4)
