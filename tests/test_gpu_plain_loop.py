"""The reference's loop body kept as it is (twotower/train.py:103-154: zero_grad, loss.backward(),
torch.optim.AdamW.step()) with the opt-in fused table update (optim.fuse_table_update, the
config's ``hip: {table_update: backward}``): the table's sorted scatter + AdamW runs at the end of
each backward, torch's AdamW steps the tower parameters.

Checked: the golden trajectory captured from the reference (3 steps incl. the decay of untouched
rows), torch.optim.AdamW's own dense-gradient update on the same weights and batches (tower and
table, at the reference's defaults), and a save_checkpoint / load_checkpoint round trip in the
middle of training that must continue the same trajectory."""
import copy
import os

import numpy as np
import pytest
import torch

import twotower_amd as tt
from twotower_amd import checkpoint, optim

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _cuda(x):
    return torch.as_tensor(np.asarray(x)).to(DEV)


def _rel(a, b):
    a = a.detach().double().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a, np.float64)
    b = b.detach().double().cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def _loop_step(model, loss_fn, opt, q, p, n):
    """train.py:120-139 (the monitors at :144-154 read the outputs only)."""
    qv, pv, nv = model(q, p, n)
    loss = loss_fn(qv, pv, nv)
    opt.zero_grad()
    loss.backward()
    opt.step()
    return float(loss.item())


@pytest.mark.parametrize("dense", [False, True])
def test_backward_table_update_trajectory_matches_reference(golden, dense):
    """dense: hip: {dense_update: backward} too (the towers' AdamW in one launch at the end of
    backward; optimizer.step() then has nothing left)."""
    g = golden("trajectory")
    V, E = g["table"].shape
    H = g["W1"].shape[0]
    emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
    model = tt.build_two_tower("mean", emb, hidden_dim=H, tied_weights=True).to(DEV)
    t = model.query_tower
    with torch.no_grad():
        for mod, k in ((t.embedding.embedding, "table"), (t.feed_forward[0], "W1"), (t.feed_forward[2], "W2")):
            mod.weight.copy_(_cuda(g[k]))
        t.feed_forward[0].bias.copy_(_cuda(g["b1"]))
        t.feed_forward[2].bias.copy_(_cuda(g["b2"]))
    opt = torch.optim.AdamW(model.parameters(), lr=float(g["lr"]))  # train.py:359
    (upd,) = optim.fuse_table_update(opt, model)
    if dense:
        optim.fuse_dense_update(opt, model)
    loss_fn = tt.losses.build("triplet", margin=0.2)
    w = t.embedding.embedding.weight
    for s in range(3):
        loss = _loop_step(model, loss_fn, opt, *(_cuda(g[f"{k}{s}"]) for k in "qpn"))
        assert w.grad is None  # the table never gets a dense gradient: torch's step skips it
        assert abs(loss - g[f"loss{s}"]) < 1e-5
        assert _rel(w, g[f"step{s}_table"]) < 1e-5
        assert _rel(t.feed_forward[0].weight, g[f"step{s}_W1"]) < 1e-5
        assert _rel(t.feed_forward[2].bias, g[f"step{s}_b2"]) < 1e-5
    assert int(opt.state[w]["step"]) == 3 and opt.state[w]["step"].device.type == "cpu"
    W1 = t.feed_forward[0].weight
    assert int(opt.state[W1]["step"]) == 3 and opt.state[W1]["step"].device.type == "cpu"
    if dense:
        assert W1.grad is None  # stepped inside backward
        opt._tt_dense_update.release()
    upd.release()
    assert not hasattr(w, "_tt_deferred")


def _model(V, E, seed):
    torch.manual_seed(seed)
    emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
    return tt.build_two_tower("mean", emb, hidden_dim=E, tied_weights=True).to(DEV)


@pytest.mark.parametrize("dense", [False, True])
@pytest.mark.parametrize("E", [128, 256])
def test_backward_table_update_equals_torch_adamw(E, dense):
    """Three loop steps at torch.optim.AdamW's defaults (lr 1e-3, wd 0.01, eps 1e-8): the fused
    table update against torch's AdamW stepping the dense table gradient of the same model (the
    planned scatter), every parameter elementwise to a few ulp + 1e-5 of lr per step; only elements
    whose gradient is within rounding of zero may differ (eps 1e-8 flips their update)."""
    V, L, B = 3001, 24, 96
    ref, fused = _model(V, E, 3), _model(V, E, 3)
    ropt = torch.optim.AdamW(ref.parameters())
    fopt = torch.optim.AdamW(fused.parameters())
    optim.fuse_table_update(fopt, fused)
    if dense:
        optim.fuse_dense_update(fopt, fused)
    loss_fn = tt.losses.build("triplet", margin=0.2)
    for s in range(3):
        if s:  # each step from the same state (the weights and moments the reference reached): an
            # eps-flipped table element would otherwise move every later gradient by rounding
            fused.load_state_dict(ref.state_dict())
            fopt.load_state_dict(copy.deepcopy(ropt.state_dict()))  # (torch's load keeps the tensors)
        batch = tt.data.synthetic_triplets(B, L, V, seed=40 + s, device=DEV)
        lr_ = _loop_step(ref, loss_fn, ropt, *batch)
        g_tab = ref.query_tower.embedding.embedding.weight.grad.detach().clone()
        lf = _loop_step(fused, loss_fn, fopt, *batch)
        assert abs(lf - lr_) < 1e-6 * max(1.0, abs(lr_)), (s, lf, lr_)
        for (k, a), (_, b) in zip(ref.named_parameters(), fused.named_parameters()):
            want, got = a.detach().double(), b.detach().double()
            tol = 1e-5 * 1e-3 + 4 * 2.0 ** -24 * want.abs()
            bad = (got - want).abs() > tol
            if bad.any():  # AdamW at eps 1e-8 amplifies gradients of order eps: only such table
                # elements, and few of them, may differ
                nb = int(bad.sum())
                assert "embedding" in k, (s, k, nb, float((got - want).abs().max()))
                assert float(g_tab[bad].abs().max()) < 1e-6 and nb <= max(4, a.numel() // 10_000), (
                    s, k, nb, float(g_tab[bad].abs().max()))
    wr, wf = ref.query_tower.embedding.embedding.weight, fused.query_tower.embedding.embedding.weight
    for key in ("exp_avg", "exp_avg_sq"):
        assert _rel(fopt.state[wf][key], ropt.state[wr][key]) < 1e-5, key
    assert int(fopt.state[wf]["step"]) == int(ropt.state[wr]["step"]) == 3


@pytest.mark.parametrize("dense", [False, True])
def test_backward_table_update_checkpoint_round_trip(tmp_path, dense):
    """save_checkpoint after two steps, load into a fresh model + torch.optim.AdamW with the fused
    table update, and the third step equals the uninterrupted run's bit for bit (the table moments
    and step counter travel in the optimizer's state_dict under torch's keys)."""
    V, E, L, B = 3001, 128, 24, 96
    batches = [tt.data.synthetic_triplets(B, L, V, seed=60 + s, device=DEV) for s in range(3)]
    loss_fn = tt.losses.build("triplet", margin=0.2)
    a = _model(V, E, 4)
    aopt = torch.optim.AdamW(a.parameters())
    optim.fuse_table_update(aopt, a)
    if dense:
        optim.fuse_dense_update(aopt, a)
    for s in range(2):
        _loop_step(a, loss_fn, aopt, *batches[s])
    path = checkpoint.save_checkpoint(a, {"<pad>": 0}, aopt, epoch=1, loss=0.5, checkpoint_dir=str(tmp_path),
                                      checkpoint_name="mid.pt", save_best=False)
    assert os.path.exists(path)
    _loop_step(a, loss_fn, aopt, *batches[2])

    b = _model(V, E, 99)  # other weights: everything must come from the checkpoint
    bopt = torch.optim.AdamW(b.parameters())
    optim.fuse_table_update(bopt, b)
    if dense:
        optim.fuse_dense_update(bopt, b)
    ck = checkpoint.load_checkpoint(path, b, bopt, device=DEV)
    assert ck["epoch"] == 1
    wb = b.query_tower.embedding.embedding.weight
    assert int(bopt.state[wb]["step"]) == 2 and bopt.state[wb]["exp_avg"].device == wb.device
    _loop_step(b, loss_fn, bopt, *batches[2])
    for (k, x), (_, y) in zip(a.named_parameters(), b.named_parameters()):
        assert torch.equal(x, y), k
