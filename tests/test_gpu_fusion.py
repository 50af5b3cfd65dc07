"""GPU: cross-kernel fusions must not change a bit.  Each fused path is compared with the unfused
launches it replaces on the same inputs (torch.equal on every output and gradient), and the test
checks that the fused entry point actually ran.

* tower head normalise pass + in-batch scorer operand prep (tt_inbatch_l2_prep, then
  tt_inbatch_fwd_prepped) against tt_head_gemm epi 1 + tt_inbatch_fwd's own prep pass."""
import numpy as np
import pytest
import torch

import twotower_amd as tt
from twotower_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(V, seed, E=256):
    torch.manual_seed(seed)
    emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
    return tt.build_two_tower("mean", emb, hidden_dim=E, tied_weights=True).to(DEV)


def _ids(B, L, V, rng):
    ids = rng.integers(1, V, size=(B, L))
    lengths = rng.integers(1, L + 1, size=B)
    ids[np.arange(L)[None, :] >= lengths[:, None]] = 0
    return torch.as_tensor(ids, device=DEV)


def _step(model, loss_fn, batch):
    model.zero_grad(set_to_none=True)
    q, p, n = model(*batch)
    loss = loss_fn(q, p, n)
    loss.backward()
    torch.cuda.synchronize()
    grads = {k: v.grad.clone() for k, v in model.named_parameters()}
    return (q.detach().clone(), p.detach().clone(), n.detach().clone(), loss.detach().clone()), grads


@pytest.mark.parametrize("B,L,dtype,bwd", [(8192, 64, "bf16", "stored"), (300, 12, "bf16", "stored"),
                                           (129, 7, "bf16", "recompute"), (256, 16, "bf16_split", "stored"),
                                           (4096, 32, "fp32", "stored"), (300, 12, "fp32", "stored"),
                                           (129, 7, "fp32", "recompute")])
def test_head_normalise_fused_with_scorer_prep_is_bit_identical(B, L, dtype, bwd, monkeypatch):
    """bf16 at H = 256 (C3) and fp32 at H = 128 (C2, l2_prep128_kernel)."""
    V = 5000
    E = 128 if dtype == "fp32" else 256
    rng = np.random.default_rng(B + L)
    batch = [_ids(B, L, V, rng) for _ in range(3)]
    loss_fn = tt.losses.build("in_batch", temperature=0.05, compute_dtype=dtype)
    assert tt.losses.scorer_prep_dtype(loss_fn) == dtype
    prev = ops.set_inbatch_backward(bwd)
    try:
        model = _model(V, 7, E)
        ref_out, ref_grads = _step(model, loss_fn, batch)

        seen = []
        real_call = ops.call

        def spy(name, *args):
            seen.append(name)
            return real_call(name, *args)

        monkeypatch.setattr(ops, "call", spy)
        model.scorer_prep = dtype
        out, grads = _step(model, loss_fn, batch)
    finally:
        ops.set_inbatch_backward(prev)
    assert "tt_inbatch_l2_prep" in seen and "tt_inbatch_fwd_prepped" in seen and "tt_inbatch_fwd" not in seen
    for a, b, name in zip(out, ref_out, ("q", "p", "n", "loss")):
        assert torch.equal(a, b), name
    for k in ref_grads:
        assert torch.equal(grads[k], ref_grads[k]), k


def test_scorer_prep_set_by_trainstep_and_ignored_by_other_losses():
    model = _model(100, 0)
    opt = tt.optim.AdamW(model.parameters(), lr=1e-3)
    st = tt.TrainStep(model, tt.losses.build("in_batch", compute_dtype="bf16"), opt)
    assert st._scorer_prep == "bf16" and model.scorer_prep is None
    seen = []
    real_call = ops.call

    def spy(name, *args):
        seen.append(name)
        return real_call(name, *args)

    rng = np.random.default_rng(3)
    batch = [_ids(64, 8, 100, rng) for _ in range(3)]
    ops.call = spy
    try:
        st(*batch)  # the prep is open for the step's own forward only
        assert "tt_inbatch_l2_prep" in seen
        assert model.scorer_prep is None
        seen.clear()
        with torch.no_grad():
            model(*batch)  # a later forward outside the step: no operand prep
        assert "tt_inbatch_l2_prep" not in seen
    finally:
        ops.call = real_call
    model2 = _model(100, 0)
    st2 = tt.TrainStep(model2, tt.losses.build("in_batch", compute_dtype="fp32"), tt.optim.AdamW(model2.parameters()))
    assert st2._scorer_prep == "fp32" and model2.scorer_prep is None
    ops.call = spy
    try:  # fp32 at H = 256: no fused prep shape, the head normalises as usual
        seen.clear()
        st2(*batch)
        assert "tt_inbatch_l2_prep" not in seen and "tt_inbatch_fwd" in seen
    finally:
        ops.call = real_call
    model3 = _model(100, 0, 128)
    st3 = tt.TrainStep(model3, tt.losses.build("in_batch", compute_dtype="fp32"), tt.optim.AdamW(model3.parameters()))
    ops.call = spy
    try:  # fp32 at H = 128 (C2): the head's normalise pass forms the scorer's norms
        seen.clear()
        st3(*batch)
        assert "tt_inbatch_l2_prep" in seen and "tt_inbatch_fwd_prepped" in seen
    finally:
        ops.call = real_call
    # a head output carrying prepared operands into a triplet loss: ignored, same loss
    model.scorer_prep = "bf16"
    trip = tt.losses.build("triplet")
    model.zero_grad(set_to_none=True)
    a = trip(*model(*batch))
    model.scorer_prep = None
    b = trip(*model(*batch))
    assert torch.equal(a, b)



def _train(model, opt, loss_fn, batches):
    for b in batches:
        opt.zero_grad(set_to_none=True)
        loss_fn(*model(*b)).backward()
        opt.step()
    torch.cuda.synchronize()
    return {k: v.detach().clone() for k, v in model.named_parameters()}


@pytest.mark.parametrize("fused_tables", [False, True])
@pytest.mark.parametrize("tied", [True, False])
def test_bag_scaling_in_head_dx_epilogue_is_bit_identical(fused_tables, tied, monkeypatch):
    """The tower head's dx GEMM divides each row by its bag denominator (tt_head_gemm epi 5) and
    the bag backward skips its scaling pass: table and head parameters after three AdamW steps
    equal the unfused launches (TT_BAG_PRESCALE=0), for the fused scatter + AdamW and for the
    dense table gradient, for the one-head TwoTower path and towers called one by one."""
    V, B, L = 3000, 200, 24
    rng = np.random.default_rng(5)
    batches = [[_ids(B, L, V, rng) for _ in range(3)] for _ in range(3)]
    loss_fn = tt.losses.build("in_batch", temperature=0.1)

    class PerTower(torch.nn.Module):  # each tower called on its own (BaseTower.forward, three bag calls)
        def __init__(self, tower):
            super().__init__()
            self.tower = tower

        def forward(self, q, p, n):
            return self.tower(q), self.tower(p), self.tower(n)

    def run():
        torch.manual_seed(3)
        emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=256)
        model = tt.build_two_tower("mean", emb, hidden_dim=256, tied_weights=True).to(DEV)
        if not tied:
            model = PerTower(model.query_tower)
        kw = dict(fused_tables=True, tables=[emb]) if fused_tables else {}
        return _train(model, tt.optim.AdamW(model.parameters(), lr=1e-3, **kw), loss_fn, batches)

    seen = []
    real_call = ops.call

    def spy(name, *args):
        seen.append((name, args[6] if name == "tt_head_gemm" else None))
        return real_call(name, *args)

    monkeypatch.setattr(ops, "call", spy)
    monkeypatch.setenv("TT_BAG_PRESCALE", "1")
    got = run()
    assert ("tt_head_gemm", 5) in seen
    monkeypatch.setenv("TT_BAG_PRESCALE", "0")
    seen.clear()
    want = run()
    assert ("tt_head_gemm", 5) not in seen
    for k in want:
        assert torch.equal(got[k], want[k]), k


@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("dtype,bwd,d,n_in", [("bf16", "stored", 256, 3), ("bf16", "recompute", 256, 3),
                                              ("bf16_split", "stored", 256, 3), ("bf16", "stored", 256, 2),
                                              ("fp32", "stored", 128, 3), ("fp32", "recompute", 128, 3),
                                              ("fp32", "stored", 128, 2)])
def test_inbatch_combine_fused_with_head_l2_backward_is_bit_identical(graph, dtype, bwd, d, n_in, monkeypatch):
    """TrainStep runs the in-batch loss's backward combine fused with the tower head's
    F.normalize backward (tt_inbatch_bwd_l2: dq, dd never written; bf16 at H = 256, fp32 at H =
    128), for the triplet form (q, p, n: M = 2B) and the pairs form (q, p: M = B); parameters and
    losses after four steps equal the unfused combine + tt_l2norm_bwd (TT_FUSED_L2_BWD=0) bit for
    bit."""
    V, B, L = 4000, 320, 20
    rng = np.random.default_rng(9)
    batches = [[_ids(B, L, V, rng) for _ in range(n_in)] for _ in range(4)]

    def run():
        torch.manual_seed(4)
        emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=d)
        model = tt.build_two_tower("mean", emb, hidden_dim=d, tied_weights=True).to(DEV)
        opt = tt.optim.AdamW(model.parameters(), lr=1e-3, fused_tables=True, tables=[emb], capturable=True)
        step = tt.TrainStep(model, tt.losses.build("in_batch", temperature=0.05, compute_dtype=dtype), opt,
                            graph=graph, eager_steps=1)
        losses = [step(*b).clone() for b in batches]
        torch.cuda.synchronize()
        return losses, {k: v.detach().clone() for k, v in model.named_parameters()}

    seen = []
    real_call = ops.call

    def spy(name, *args):
        seen.append(name)
        return real_call(name, *args)

    prev = ops.set_inbatch_backward(bwd)
    try:
        monkeypatch.setattr(ops, "call", spy)
        got_l, got = run()
        assert "tt_inbatch_bwd_l2" in seen and "tt_l2norm_bwd" not in seen
        monkeypatch.setenv("TT_FUSED_L2_BWD", "0")
        seen.clear()
        want_l, want = run()
        assert "tt_inbatch_bwd_l2" not in seen and "tt_l2norm_bwd" in seen
    finally:
        ops.set_inbatch_backward(prev)
    for a, b in zip(got_l, want_l):
        assert torch.equal(a, b)
    for k in want:
        assert torch.equal(got[k], want[k]), k


@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("K", [1, 4, 7])
def test_multi_neg_fused_with_head_l2_backward_is_bit_identical(graph, K, monkeypatch):
    """TrainStep runs the multiple-negatives loss backward fused with the tower head's F.normalize
    backward (tt_multi_neg_bwd_l2, H = 256: the loss writes the gradient before F.normalize, the
    head skips tt_l2norm_bwd); parameters and losses after four steps equal the two launches
    (TT_FUSED_L2_BWD=0) bit for bit, for 1, 4 and 7 negatives per query (C5: 4)."""
    V, B, L, d = 4000, 160, 20, 256
    rng = np.random.default_rng(11 + K)
    batches = [[_ids(B, L, V, rng), _ids(B, L, V, rng), _ids(B * K, L, V, rng)] for _ in range(4)]

    def run():
        torch.manual_seed(5)
        emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=d)
        model = tt.build_two_tower("mean", emb, hidden_dim=d, tied_weights=True).to(DEV)
        opt = tt.optim.AdamW(model.parameters(), lr=1e-3, fused_tables=True, tables=[emb], capturable=True)
        mn = tt.losses.build("multiple_negatives", temperature=0.1)

        def loss_fn(q, p, n):  # negatives viewed (B, K, H), as bench.py's C5 line feeds them
            return mn(q, p, n.view(q.shape[0], K, q.shape[1]))

        step = tt.TrainStep(model, loss_fn, opt, graph=graph, eager_steps=1)
        losses = [step(*b).clone() for b in batches]
        torch.cuda.synchronize()
        return losses, {k: v.detach().clone() for k, v in model.named_parameters()}

    seen = []
    real_call = ops.call

    def spy(name, *args):
        seen.append(name)
        return real_call(name, *args)

    monkeypatch.setattr(ops, "call", spy)
    got_l, got = run()
    assert "tt_multi_neg_bwd_l2" in seen and "tt_l2norm_bwd" not in seen
    monkeypatch.setenv("TT_FUSED_L2_BWD", "0")
    seen.clear()
    want_l, want = run()
    assert "tt_multi_neg_bwd_l2" not in seen and "tt_l2norm_bwd" in seen
    for a, b in zip(got_l, want_l):
        assert torch.equal(a, b)
    for k in want:
        assert torch.equal(got[k], want[k]), k


@pytest.mark.parametrize("E,H", [(256, 256), (128, 128), (64, 128), (128, 256)])
def test_bag_forward_split_workgroups_equal_head_split(E, H):
    """tt_bag_mean_fwd_split: the pooled rows and denominators equal tt_bag_mean_fwd's and the
    planes equal tt_head_split_ff2's, bit for bit (one and 37 sequences)."""
    rng = np.random.default_rng(E + H)
    V = 700
    table = torch.randn(V, E, device=DEV)
    W1, W2 = torch.randn(H, E, device=DEV), torch.randn(H, H, device=DEV)
    n1, n2 = ops._head_planes_bytes(E, H)
    for B in (37, 1):
        ids = _ids(B, 9, V, rng).to(torch.int32)
        ref_p, ref_d = ops.bag_mean_forward(table, ids)
        ref_planes = torch.empty(2 * (n1 + n2), dtype=torch.uint8, device=DEV)
        ops.call("tt_head_split_ff2", ops.ptr(W1), ops.ptr(W2), E, H, ops.ptr(ref_planes), ops.stream_of(W1))
        with ops.head_planes_in_gather(W1, W2):
            p, d = ops.bag_mean_forward(table, ids)
            planes = ops._PLANES_DONE[(W1.data_ptr(), W2.data_ptr())]
        torch.cuda.synchronize()
        assert not ops._PLANES_DONE
        assert torch.equal(p, ref_p) and torch.equal(d, ref_d)
        assert torch.equal(planes, ref_planes)


@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("tied,H", [(True, 256), (False, 256), (True, 128)])
def test_head_planes_formed_in_gather_are_bit_identical(graph, tied, H, monkeypatch):
    """The gather's launch forms the head's weight planes (ops.head_planes_in_gather): losses and
    parameters after four TrainSteps (eager, and graph replays after one eager step) equal the
    in-line split (TT_PLANES_IN_GATHER=0); the head takes them (no tt_head_split_ff2 launch on the
    tied path; the untied towers pool and split as before)."""
    V, B, L = 3000, 256, 24
    rng = np.random.default_rng(11)
    batches = [[_ids(B, L, V, rng) for _ in range(3)] for _ in range(4)]

    def run():
        torch.manual_seed(5)
        emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=H)
        model = tt.build_two_tower("mean", emb, hidden_dim=H, tied_weights=tied).to(DEV)
        opt = tt.optim.AdamW(model.parameters(), lr=1e-3, fused_tables=True, tables=[emb], capturable=True)
        st = tt.TrainStep(model, tt.losses.build("in_batch", temperature=0.1, compute_dtype="bf16"), opt,
                          graph=graph, eager_steps=1)
        losses = [st(*b).clone() for b in batches]
        torch.cuda.synchronize()
        return losses, {k: v.detach().clone() for k, v in model.named_parameters()}

    seen = []
    real_call = ops.call

    def spy(name, *args):
        seen.append(name)
        return real_call(name, *args)

    monkeypatch.setattr(ops, "call", spy)
    monkeypatch.setenv("TT_PLANES_IN_GATHER", "1")
    got_l, got = run()
    if tied:
        assert "tt_bag_mean_fwd_split" in seen and "tt_head_split_ff2" not in seen
    assert not ops._PLANES_DONE and not ops._PLANES_REQ
    monkeypatch.setenv("TT_PLANES_IN_GATHER", "0")
    seen.clear()
    want_l, want = run()
    assert "tt_bag_mean_fwd_split" not in seen
    for a, b in zip(got_l, want_l):
        assert torch.equal(a, b)
    for k in want:
        assert torch.equal(got[k], want[k]), k


def test_single_tower_forward_takes_planes_from_its_gather():
    """BaseTower.forward of a hand-written-head MeanPoolingTower (a tower called on its own):
    one tt_bag_mean_fwd_split, no tt_head_split_ff2, same output and gradients as the in-line split."""
    torch.manual_seed(2)
    emb = tt.embeddings.build("lookup", vocab_size=500, embedding_dim=256)
    tower = tt.build_two_tower("mean", emb, hidden_dim=256, tied_weights=True).to(DEV).query_tower
    ids = _ids(40, 10, 500, np.random.default_rng(4))
    seen = []
    real_call = ops.call

    def spy(name, *args):
        seen.append(name)
        return real_call(name, *args)

    outs = []
    for on in ("1", "0"):
        import os
        os.environ["TT_PLANES_IN_GATHER"] = on
        try:
            ops.call = spy
            tower.zero_grad(set_to_none=True)
            y = tower(ids)
            y.square().sum().backward()
        finally:
            ops.call = real_call
            os.environ.pop("TT_PLANES_IN_GATHER")
        outs.append((y.detach().clone(), {k: v.grad.clone() for k, v in tower.named_parameters()}))
        if on == "1":
            assert "tt_bag_mean_fwd_split" in seen and "tt_head_split_ff2" not in seen
    assert torch.equal(outs[0][0], outs[1][0])
    for k in outs[1][1]:
        assert torch.equal(outs[0][1][k], outs[1][1][k]), k
