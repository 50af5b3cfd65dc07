"""GPU parity at the bench's full sizes (BASELINE.json configs[2], C3: V 200k, E = H 256, L 64,
B 8192 queries + their positive and negative documents), through checks that do not need the
oracle to process the whole batch: exact identities (denominators, single-token bags, the fused
update against the unfused path bit for bit, graph replay against eager), the float64 oracle on
sampled rows, and the bf16 scorer against a plain PyTorch float64 computation on the same
bf16-rounded operands.  Each test runs in a few seconds."""
import numpy as np
import pytest
import torch

import twotower_amd as tt
from twotower_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"
V, E, L, B = 200_000, 256, 64, 8192


def _ids(seed=0):
    q, p, n = tt.data.synthetic_triplets(B, L, V, seed=seed, device=DEV)
    ids = torch.cat([q, p, n]).contiguous()
    ids[5] = 0                    # an all-pad sequence
    ids[6, 1:] = 0                # single-token sequences
    ids[7, 1:] = 0
    ids[7, 0] = V - 1             # ... of the last row
    ids[8, 3] = 0                 # an interior pad
    return ids


def _rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def test_c3_bag_forward_full_size():
    torch.manual_seed(0)
    table = torch.randn(V, E, device=DEV)
    ids = _ids()
    pooled, denom = ops.bag_mean_forward(table, ids)
    cnt = (ids > 0).sum(1).float()
    assert torch.equal(denom, cnt + 1e-9)                                 # encoders.py:72, fp32
    assert torch.count_nonzero(pooled[5]) == 0
    assert torch.equal(pooled[6], table[ids[6, 0]]) and torch.equal(pooled[7], table[V - 1])  # bit-exact
    rows = np.random.default_rng(1).choice(ids.shape[0], 256, replace=False)
    ids_h = ids[rows].cpu().numpy()
    tab = table.double().cpu().numpy()
    want = np.stack([tab[r[r > 0]].sum(0) / max((r > 0).sum(), 1e-9) for r in ids_h])
    assert _rel(pooled[rows].double().cpu().numpy(), want) < 1e-6


def test_c3_fused_update_full_size_equals_unfused_and_oracle():
    """The fused scatter + AdamW (XCD-sliced reduce) equals the dense-gradient path + AdamW
    bit for bit over two steps at C3 size; the dense gradient matches the float64 oracle on
    sampled rows (hot and cold)."""
    torch.manual_seed(1)
    ids = _ids(seed=2)
    t0 = torch.randn(V, E, device=DEV)
    d_pooled = torch.randn(ids.shape[0], E, device=DEV)
    _, denom = ops.bag_mean_forward(t0, ids)
    A, Bt = t0.clone(), t0.clone()
    mA, vA, mB, vB = (torch.zeros_like(t0) for _ in range(4))
    hp = dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01)
    for step in (1, 2):
        grad = ops.bag_mean_backward(d_pooled, denom, ids, V, 0)
        ops.adamw_step(A, grad, mA, vA, step=step, **hp)
        ops.bag_mean_backward_adamw(d_pooled, denom, ids, Bt, mB, vB, 0, step=step, **hp)
    assert torch.equal(A, Bt) and torch.equal(mA, mB) and torch.equal(vA, vB)
    # oracle on sampled rows: G[r] = sum over tokens t with id r of d_pooled[seq(t)] / denom[seq(t)]
    ids_h = ids.cpu().numpy()
    counts = np.bincount(ids_h.ravel(), minlength=V)
    hot = np.argsort(counts[1:])[-4:] + 1
    rows = np.concatenate([hot, np.random.default_rng(3).choice(np.arange(1, V), 60, replace=False), [0]])
    gs = (d_pooled.double() / denom.double()[:, None]).cpu().numpy()
    want = np.zeros((len(rows), E))
    for k, r in enumerate(rows):
        if r == 0:
            continue                                                     # padding row: no gradient
        seqs, _ = np.nonzero(ids_h == r)
        want[k] = gs[seqs].sum(0)
    got = grad[torch.as_tensor(rows, device=DEV)].double().cpu().numpy()
    assert _rel(got, want) < 1e-5
    assert not got[-1].any()


def _ref64_in_batch(q, d, tau, off, g=1.0):
    """in_batch_sampled_softmax_loss (twotower/losses.py:88-118) in float64 on the GPU (plain
    PyTorch: the oracle's formula at a size the host would take minutes for)."""
    z = (q.double() @ d.double().T) / tau
    B = q.shape[0]
    rows = torch.arange(B, device=DEV)
    lse = torch.logsumexp(z, 1)
    loss = (lse - z[rows, rows + off]).mean()
    P = torch.exp(z - lse[:, None])
    del z
    P[rows, rows + off] -= 1.0
    P *= g / B
    return loss.item(), (P @ d.double()) / tau, (P.T @ q.double()) / tau


def _rel_t(a, b):
    return float((a.double() - b).abs().max() / b.abs().max())


# Measured errors (tools/scorer_error_table.py --big, profiles/r02_scorer_error.md) against float64
# on the bf16-rounded operands; the bars below are about 1.5-2x those:
#   C3 (B 8192, M 16384): stored bf16 dq 1.64e-5 dd 1.54e-5; bf16_split dq 7.9e-8 dd 7.1e-8
#   C4 rank (M 131072):   stored bf16 dq 5.5e-6  dd 2.0e-6;  bf16_split dq 9.3e-8 dd 7.1e-8
@pytest.mark.parametrize("form,tol", [("bf16", 3e-5), ("bf16_split", 1.5e-7)])
def test_c3_scorer_full_size_vs_fp64(form, tol):
    """The bf16 scorer forms at B 8192 x M 16384 x H 256 (C3, M = 2B) against float64 on the same
    bf16-rounded q, d: loss to 1e-6, gradients to about 1.5-2x the measured error."""
    g = torch.Generator(device=DEV).manual_seed(4)
    q = torch.nn.functional.normalize(torch.randn(B, E, device=DEV, generator=g), dim=-1)
    d = torch.nn.functional.normalize(torch.randn(2 * B, E, device=DEV, generator=g), dim=-1)
    Q, D = q.clone().requires_grad_(True), d.clone().requires_grad_(True)
    loss = ops.in_batch_softmax_loss(Q, D, 0.1, compute_dtype=form)
    loss.backward()
    rl, rdq, rdd = _ref64_in_batch(q.bfloat16().float(), d.bfloat16().float(), 0.1, 0)
    assert abs(loss.item() - rl) < 1e-6 * abs(rl)
    assert _rel_t(Q.grad, rdq) < tol and _rel_t(D.grad, rdd) < tol


@pytest.mark.parametrize("per_rank", [2, 1])
def test_c4_rank_scorer_at_eight_gpu_shape_vs_fp64(per_rank):
    """One rank of the 8-GPU cross-device step (BASELINE.json configs[3], C4): its B 8192 queries
    against all gathered candidates, labels offset to rank 5's block, H 256, on the bf16 scorer
    (stored probabilities), against float64 on the same bf16-rounded operands: loss to 1e-6,
    gradients to 1e-5 (measured 5.5e-6 / 2.0e-6 in the triplet form).  per_rank 2: the triplet
    form, 8 x 2B = 131072 candidates (2 GiB of P); per_rank 1: the pairs form as configs[3]
    states it, 8 x B = 65536 global negatives (bench.py's c4_pairs entry)."""
    world, rank = 8, 5
    M = world * per_rank * B
    g = torch.Generator(device=DEV).manual_seed(9)
    q = torch.nn.functional.normalize(torch.randn(B, E, device=DEV, generator=g), dim=-1)
    d = torch.nn.functional.normalize(torch.randn(M, E, device=DEV, generator=g), dim=-1)
    Q, D = q.clone().requires_grad_(True), d.clone().requires_grad_(True)
    off = rank * per_rank * B
    loss = ops.in_batch_softmax_loss(Q, D, 0.1, label_off=off, compute_dtype="bf16")
    loss.backward()
    rl, rdq, rdd = _ref64_in_batch(q.bfloat16().float(), d.bfloat16().float(), 0.1, off)
    assert abs(loss.item() - rl) < 1e-6 * abs(rl)
    assert _rel_t(Q.grad, rdq) < 1e-5 and _rel_t(D.grad, rdd) < 1e-5
    # candidates of other ranks' blocks receive only softmax mass: no label term there
    assert float(D.grad[:off].abs().max()) < float(D.grad[off:off + B].abs().max())


def test_c3_step_graph_equals_eager_full_size():
    """Two C3 training steps (fused towers, bf16 in-batch loss over 2B candidates, fused table
    AdamW, side-stream plan and weight gradients): graph replay equals eager bit for bit."""

    def build():
        torch.manual_seed(5)
        emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
        model = tt.build_two_tower("mean", emb, hidden_dim=E, tied_weights=True).to(DEV)
        opt = tt.optim.AdamW(model.parameters(), lr=1e-3, fused_tables=True, tables=[emb], capturable=True)
        return model, opt, tt.losses.build("in_batch", temperature=0.1, compute_dtype="bf16")

    batches = [tt.data.synthetic_triplets(B, L, V, seed=10 + k, device=DEV) for k in range(3)]
    m1, o1, l1 = build()
    s1 = tt.TrainStep(m1, l1, o1)
    losses = [s1(*b).item() for b in batches]
    p1 = [p.detach().clone() for p in m1.parameters()]
    del s1, o1, m1
    m2, o2, l2 = build()
    s2 = tt.TrainStep(m2, l2, o2, graph=True, eager_steps=1)
    for b, want in zip(batches, losses):
        assert s2(*b).item() == want
    assert len(s2._graphs) == 1
    for a, b_ in zip(p1, m2.parameters()):
        assert torch.equal(a, b_)
    assert np.isfinite(losses).all() and losses[0] > losses[-1] - 1.0


def test_c5_full_size_update_and_multi_negative_loss():
    """C5 shape (configs[4] per GPU: V 1M, 8192 queries x (1 positive + 4 negatives)): the fused
    update equals the unfused path bit for bit, and multiple_negatives matches a plain PyTorch
    fp32/fp64 restatement of losses.py:47-85 (loss and gradients 1e-5)."""
    Vc, K = 1_000_000, 4
    q, p, n = tt.data.synthetic_triplets(B, L, Vc, seed=6, device=DEV, negatives=K)
    ids = torch.cat([q, p, n]).contiguous()
    assert ids.shape == ((2 + K) * B, L)
    torch.manual_seed(7)
    t0 = torch.randn(Vc, E, device=DEV)
    d_pooled = torch.randn(ids.shape[0], E, device=DEV)
    _, denom = ops.bag_mean_forward(t0, ids)
    A, Bt = t0.clone(), t0.clone()
    mA, vA, mB, vB = (torch.zeros_like(t0) for _ in range(4))
    hp = dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01)
    grad = ops.bag_mean_backward(d_pooled, denom, ids, Vc, 0)
    ops.adamw_step(A, grad, mA, vA, step=1, **hp)
    ops.bag_mean_backward_adamw(d_pooled, denom, ids, Bt, mB, vB, 0, step=1, **hp)
    assert torch.equal(A, Bt) and torch.equal(mA, mB) and torch.equal(vA, vB)
    del A, Bt, mA, vA, mB, vB, grad, t0

    g = torch.Generator(device=DEV).manual_seed(8)
    qv, pv, nv = (torch.randn(r, E, device=DEV, generator=g) for r in (B, B, K * B))
    Q, P, N = (x.clone().requires_grad_(True) for x in (qv, pv, nv))
    loss = tt.losses.multiple_negatives_loss(Q, P, N.view(B, K, E), temperature=0.1)
    loss.backward()
    Qr, Pr, Nr = (x.double().requires_grad_(True) for x in (qv, pv, nv))
    docs = torch.cat([Pr.unsqueeze(1), Nr.view(B, K, E)], 1)
    logits = torch.nn.functional.cosine_similarity(Qr.unsqueeze(1).expand_as(docs), docs, dim=2) / 0.1
    ref = torch.nn.functional.cross_entropy(logits, torch.zeros(B, dtype=torch.long, device=DEV))
    ref.backward()
    assert abs(loss.item() - ref.item()) < 1e-5 * abs(ref.item())
    for got, want in ((Q.grad, Qr.grad), (P.grad, Pr.grad), (N.grad, Nr.grad)):
        assert _rel(got.double().cpu().numpy(), want.cpu().numpy()) < 1e-5


# ---------------------------------------------------------------------------------------------
# C2 (BASELINE.json configs[1]): V 50k, d 128, L 32, B 4096, in-batch negatives over M = 2B, fp32
V2, E2, L2, B2 = 50_000, 128, 32, 4096


def test_c2_scorer_full_size_vs_fp64_oracle():
    """The fp32 in-batch scorer at the C2 shape (B 4096 queries x M 8192 candidates, H 128)
    against the float64 oracle restatement of losses.py:88-118 (oracle/reference_math.py) on the
    whole batch: loss, dq and dd within 1e-5 (max-abs normalised)."""
    from oracle import reference_math as O

    g = torch.Generator(device=DEV).manual_seed(21)
    q = torch.nn.functional.normalize(torch.randn(B2, E2, device=DEV, generator=g), dim=-1)
    d = torch.nn.functional.normalize(torch.randn(2 * B2, E2, device=DEV, generator=g), dim=-1)
    Q, D = q.clone().requires_grad_(True), d.clone().requires_grad_(True)
    loss = tt.losses.in_batch_sampled_softmax_loss(Q, D, temperature=0.1, compute_dtype="fp32")
    loss.backward()
    rl, (rdq, rdd), _ = O.in_batch_fwd_bwd(q.double().cpu().numpy(), d.double().cpu().numpy(), 0.1)
    assert abs(loss.item() - rl) < 1e-5 * abs(rl)
    assert _rel(Q.grad.double().cpu().numpy(), rdq) < 1e-5
    assert _rel(D.grad.double().cpu().numpy(), rdd) < 1e-5


def test_c2_step_full_size_at_reference_settings():
    """A whole C2 training step (3 x 4096 sequences of 32 ids over a 50k x 128 table, tied
    Linear-ReLU-Linear tower, fp32 in-batch loss over cat[p, n]) at the reference's AdamW
    settings (eps 1e-8, weight decay 0.01; twotower/train.py:359): the HIP gradients (loss, the
    dense table gradient, every head gradient) against the float64 restatement of the reference
    step within 1e-5, and the fused table update of a graph-replayed TrainStep against
    torch.optim.AdamW on those gradients, elementwise (tests/_step_parity.py)."""
    import _step_parity

    r = _step_parity.run(V2, E2, L2, B2, "in_batch", "fp32", grad_tol=1e-5, seed=22, graph=True)
    print(r)


def test_c3_step_full_size_at_reference_settings():
    """The C3 training step (V 200k, d 256, L 64, B 8192, bf16 in-batch scorer over 2B
    candidates) at the reference's AdamW settings: the loss within 1e-5; the scorer's operand
    gradients against float64 on the same bf16-rounded operands at 2e-4 (measured on these
    operands, the step's own tower outputs: q 4.3e-5, p 3.0e-5, n 7.7e-5; the suite's general
    bf16 bar is 2e-3); every parameter gradient against the float64 towers driven by those HIP
    operand gradients at 1e-5 (measured <= 1.9e-6); then the fused update of a graph-replayed
    TrainStep against torch.optim.AdamW on the HIP gradients, elementwise."""
    import _step_parity

    r = _step_parity.run(V, E, L, B, "in_batch", "bf16", grad_tol=2e-4, seed=23, graph=True)
    print(r)
