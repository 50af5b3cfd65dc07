"""The optimizer's fused tail (tt_adamw_multi_ex): the head weight gradients' slab sums, the
dense AdamW updates and the next step's scalars in one launch, against the three launches it
replaces (tt_head_wgrad2_reduce, tt_adamw_multi, tt_adam_prepare_ex(1, 1)) -- bit for bit, as
the kernel, and through TrainStep (TT_FUSED_TAIL=0 selects the three launches).  Also the
step's head: the batch copied into the replayed graph's packed input by tt_pack_blocks."""
import numpy as np
import pytest
import torch

import twotower_amd as tt
from twotower_amd import _lib, ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _state(shape, rng):
    p = torch.as_tensor(rng.standard_normal(shape).astype(np.float32)).to(DEV)
    m = torch.as_tensor(rng.standard_normal(shape).astype(np.float32) * 0.1).to(DEV)
    v = torch.as_tensor(np.abs(rng.standard_normal(shape)).astype(np.float32) * 0.01).to(DEV)
    return p, m, v


@pytest.mark.parametrize("rows", [96, 4096])
def test_adamw_multi_ex_equals_reduce_update_prepare(rows):
    rng = np.random.default_rng(7 + rows)
    mats = [torch.as_tensor(rng.standard_normal((rows, 256)).astype(np.float32)).to(DEV) for _ in range(4)]
    ws = ops.head_wgrad2(*mats)
    shapes = [(256, 256), (256,), (256, 256), (256,)]
    hyper = dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01)
    runs = []
    for fused in (False, True):
        r = np.random.default_rng(3)
        params = [_state(s, r) for s in shapes]
        grads = [torch.full(s, float("nan"), device=DEV) for s in shapes]
        # an extra plain tensor (its own gradient, no partials) rides in the same launch
        extra = _state((1000,), r)
        extra_g = torch.as_tensor(r.standard_normal(1000).astype(np.float32)).to(DEV)
        steps = [torch.full((), 4.0, device=DEV) for _ in range(5)]
        args = [torch.zeros(8, device=DEV) for _ in range(5)]
        slots = list(zip(steps, args))
        ops.adam_prepare(slots, increment=0, ahead=1, **hyper)
        items = [(p, g, m, v, a) for (p, m, v), g, a in zip(params, grads, args)]
        items.append((extra[0], extra_g, extra[1], extra[2], args[4]))
        if fused:
            sums = ops._Wgrad2Sums(ws, [p for p, _, _ in params]).grad_parts()
            parts = [sums[id(p)] for p, _, _ in params] + [None]
            ticket = torch.zeros(_lib.TT_ADAM_TICKET_WORDS, dtype=torch.int32, device=DEV)
            ops.adamw_multi_ex(items, parts, slots, ticket=ticket, **hyper)
            torch.cuda.synchronize()
            assert not bool(ticket.any())  # left zeroed for the next launch
        else:
            ops.head_wgrad2_reduce(ws, *grads)
            ops.adamw_multi(items)
            ops.adam_prepare(slots, increment=1, ahead=1, **hyper)
        torch.cuda.synchronize()
        runs.append([t.clone() for it in items for t in it[:4]] + [t.clone() for sl in slots for t in sl])
    for a, b in zip(*runs):
        assert torch.equal(a, b)
    assert all(float(s) == 5.0 for s in runs[1][-10::2])


@pytest.mark.parametrize("sizes", [(1000,), (1000, 3000, 50), (1000,) * 5, (70000, 5, 9)])
def test_adamw_multi_ex_ticket_any_grid(sizes):
    """The two-level last-workgroup ticket on grids of 2, 8, 10 and 74 workgroups (fewer than,
    equal to and not a multiple of its eight groups; odd sizes take the scalar tail): the update
    and the next scalars equal the separate launches, and the nine ticket words are left zeroed
    for the next launch."""
    hyper = dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01)
    runs = []
    for fused in (False, True):
        r = np.random.default_rng(11)
        items, slots = [], []
        for n in sizes:
            p, m, v = _state((n,), r)
            g = torch.as_tensor(r.standard_normal(n).astype(np.float32)).to(DEV)
            st, a = torch.full((), 2.0, device=DEV), torch.zeros(8, device=DEV)
            ops.adam_prepare([(st, a)], increment=0, ahead=1, **hyper)
            items.append((p, g, m, v, a))
            slots.append((st, a))
        ticket = torch.zeros(_lib.TT_ADAM_TICKET_WORDS, dtype=torch.int32, device=DEV)
        for _ in range(3):  # the ticket is reused across launches
            if fused:
                ops.adamw_multi_ex(items, None, slots, ticket=ticket, **hyper)
            else:
                ops.adamw_multi(items)
                ops.adam_prepare(slots, increment=1, ahead=1, **hyper)
        torch.cuda.synchronize()
        assert not bool(ticket.any())
        runs.append([t.clone() for it in items for t in it[:4]] + [t.clone() for sl in slots for t in sl])
    for a, b in zip(*runs):
        assert torch.equal(a, b)
    assert all(float(s) == 5.0 for s in runs[1][-2 * len(sizes)::2])


def test_adamw_multi_ex_prepare_only():
    """No tensors, only the next step's scalars (a launch of one workgroup)."""
    hyper = dict(lr=2e-3, beta1=0.8, beta2=0.99, eps=1e-6, weight_decay=0.1)
    out = []
    for fused in (False, True):
        st, a = torch.full((), 2.0, device=DEV), torch.zeros(8, device=DEV)
        if fused:
            ops.adamw_multi_ex([], None, [(st, a)], ticket=torch.zeros(_lib.TT_ADAM_TICKET_WORDS, dtype=torch.int32, device=DEV), **hyper)
        else:
            ops.adam_prepare([(st, a)], increment=1, ahead=1, **hyper)
        torch.cuda.synchronize()
        out.append((st.clone(), a.clone()))
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])


@pytest.mark.parametrize("graph", [False, True])
def test_trainstep_fused_tail_equals_three_launches(graph, monkeypatch):
    V, E, B, L = 4000, 256, 128, 16

    def run():
        torch.manual_seed(13)
        emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
        model = tt.build_two_tower("mean", emb, hidden_dim=E, tied_weights=True).to(DEV)
        opt = tt.optim.AdamW(model.parameters(), lr=1e-3, fused_tables=True, tables=[emb], capturable=True)
        step = tt.TrainStep(model, tt.losses.build("in_batch", temperature=0.1, compute_dtype="bf16"), opt,
                            graph=graph, eager_steps=2)
        losses = [step(*tt.data.synthetic_triplets(B, L, V, seed=70 + k, device=DEV)).clone() for k in range(5)]
        torch.cuda.synchronize()
        return (losses, [p.detach().clone() for p in model.parameters()],
                [p.grad.clone() for p in model.parameters() if p.grad is not None],
                [opt.state[p]["step"].item() for p in model.parameters()])

    monkeypatch.setenv("TT_FUSED_TAIL", "1")
    got = run()
    monkeypatch.setenv("TT_FUSED_TAIL", "0")
    want = run()
    for a, b in zip(got[0], want[0]):
        assert torch.equal(a, b)
    for a, b in zip(got[1], want[1]):
        assert torch.equal(a, b)
    assert len(got[2]) == len(want[2]) >= 4
    for a, b in zip(got[2], want[2]):
        assert torch.equal(a, b)
    assert got[3] == want[3] == [5.0] * len(got[3])


@pytest.mark.parametrize("dtype,rows", [(torch.int32, (96, 96, 96)), (torch.int64, (5, 7, 3)), (torch.uint8, (3, 1, 5))])
def test_pack_blocks_equals_cat(dtype, rows):
    L = 13 if dtype == torch.uint8 else 64
    g = torch.Generator().manual_seed(5)
    srcs = [torch.randint(0, 100, (r, L), generator=g).to(dtype).to(DEV) for r in rows]
    if dtype == torch.uint8:  # an unaligned source: the byte path
        srcs[1] = torch.randint(0, 100, (rows[1] * L + 1,), generator=g).to(dtype).to(DEV)[1:].view(rows[1], L)
    dst = torch.full((sum(rows), L), 77, dtype=dtype, device=DEV)
    ops.pack_blocks(srcs, dst)
    torch.cuda.synchronize()
    assert torch.equal(dst, torch.cat(srcs, 0))


@pytest.mark.parametrize("dt", ["bf16", "fp32"])
@pytest.mark.parametrize("graph,B", [(False, 300), (True, 300), (True, 9000)])
def test_trainstep_deferred_loss_mean_equals_own_launch(graph, B, dt, monkeypatch):
    """The loss mean formed by the backward combine's extra workgroup (tt_inbatch_bwd_l2, or
    tt_inbatch_bwd when the L2 backward is not fused) equals tt_mean's launch bit for
    bit, and so does everything after it.  B 300: short strided tails; B 9000: past 8 x 1024
    rows, the eight-load loop."""
    V, L = 3000, 12
    E = 256 if dt == "bf16" else 128

    def run():
        torch.manual_seed(17)
        emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
        model = tt.build_two_tower("mean", emb, hidden_dim=E, tied_weights=True).to(DEV)
        opt = tt.optim.AdamW(model.parameters(), lr=1e-3, fused_tables=True, tables=[emb], capturable=True)
        step = tt.TrainStep(model, tt.losses.build("in_batch", temperature=0.05, compute_dtype=dt), opt,
                            graph=graph, eager_steps=2)
        losses = [step(*tt.data.synthetic_triplets(B, L, V, seed=40 + k, device=DEV)).clone() for k in range(4)]
        torch.cuda.synchronize()
        return losses, [p.detach().clone() for p in model.parameters()]

    monkeypatch.setenv("TT_DEFER_MEAN", "1")
    got = run()
    monkeypatch.setenv("TT_DEFER_MEAN", "0")
    want = run()
    assert all(bool(torch.isfinite(x)) for x in got[0])
    for a, b in zip(got[0], want[0]):
        assert torch.equal(a, b)
    for a, b in zip(got[1], want[1]):
        assert torch.equal(a, b)



@pytest.mark.parametrize("graph", [False, True])
def test_trainstep_wrapped_in_batch_loss_returns_its_value(graph):
    """A loss_fn that wraps the in-batch loss (here 0.5 x it) reads the loss value inside the
    forward: TrainStep must not defer its mean to the backward then (the value was
    uninitialised memory).  Every returned loss equals 0.5 x the loss of a no-grad forward on the
    same weights and batch, taken right before the step."""
    V, L, B, E = 3000, 12, 300, 256
    torch.manual_seed(5)
    emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
    model = tt.build_two_tower("mean", emb, hidden_dim=E, tied_weights=True).to(DEV)
    opt = tt.optim.AdamW(model.parameters(), lr=1e-3, fused_tables=True, tables=[emb], capturable=True)
    bare = tt.losses.build("in_batch", temperature=0.1, compute_dtype="bf16")
    step = tt.TrainStep(model, lambda q, p, n: 0.5 * bare(q, p, n), opt, graph=graph, eager_steps=1)
    assert not step._defer_mean
    for k in range(4):
        batch = tt.data.synthetic_triplets(B, L, V, seed=60 + k, device=DEV)
        with torch.no_grad():
            want = 0.5 * bare(*model(*batch))
        got = step(*batch).clone()
        torch.cuda.synchronize()
        assert torch.isfinite(got)
        torch.testing.assert_close(got, want, rtol=1e-6, atol=0)
