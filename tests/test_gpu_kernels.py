"""GPU parity: every HIP kernel (called through the C ABI via twotower_amd.ops) against the CPU
oracle and the reference's golden vectors.  Tolerances: token-id indexing bit-exact (gathered
rows / pooled values of single-token bags), fp32 loss and gradients within 1e-5 relative
(max-abs normalised), bf16 scorer against the oracle on bf16-rounded inputs: 1e-4 for the
hi/lo split of P (bf16_split) and the standard single-rounding bf16 form at about 1.5x their
measured errors (BF16_SPLIT_GRAD_TOL, BF16_GRAD_TOL below)."""
import ctypes
import os

import numpy as np
import pytest
import torch

import twotower_amd as tt
from twotower_amd import _lib, ops
from oracle import reference_math as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
# bf16 scorer gradient bars against the float64 oracle on the bf16-rounded operands (max-abs
# normalised), at about 1.5x the largest error `tools/scorer_error_table.py --tests` measured
# over every shape below, three seeds each (profiles/r02_scorer_error.md): stored-P bf16 1.40e-3
# (recompute 0.95e-3; B 129, M 129, H 32: few terms per sum), bf16_split 1.54e-6
BF16_GRAD_TOL = 2e-3
BF16_SPLIT_GRAD_TOL = 2.5e-6


def rel(a, b):
    a = a.detach().double().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a, np.float64)
    b = b.detach().double().cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def cuda(x, dtype=None):
    t = torch.as_tensor(np.asarray(x))
    return t.to(DEV, dtype=dtype) if dtype is not None else t.to(DEV)


def edge_ids(N, L, V, rng, dtype=torch.int64):
    ids = rng.integers(1, V, size=(N, L))
    lengths = rng.integers(0, L + 1, size=N)
    ids[np.arange(L)[None, :] >= lengths[:, None]] = 0
    if N > 3:
        ids[0, :] = 0                        # all padding
        ids[1, ::3] = 0                      # interior zeros
        ids[2, :] = V - 1                    # last row, repeated
        ids[3, : min(L, 5)] = 1
    return cuda(ids, dtype)


# ---------------------------------------------------------------------------------------------
# bag forward / backward
@pytest.mark.parametrize("E", [16, 64, 128, 256, 512, 100])
@pytest.mark.parametrize("L,dtype", [(12, torch.int64), (64, torch.int32), (100, torch.int64), (1, torch.int32)])
def test_bag_forward_vs_oracle(E, L, dtype):
    rng = np.random.default_rng(E * 1000 + L)
    V, N = 997, 203
    table = rng.standard_normal((V, E)).astype(np.float32)
    ids = edge_ids(N, L, V, rng, dtype)
    pooled, denom = ops.bag_mean_forward(cuda(table), ids)
    ref, ref_den = O.bag_mean_fwd(table.astype(np.float64), ids.cpu().numpy())
    assert rel(pooled, ref) < 1e-5
    np.testing.assert_allclose(denom.cpu().numpy(), ref_den.astype(np.float32), rtol=0, atol=0)
    assert torch.count_nonzero(pooled[0]) == 0


def test_bag_forward_gather_is_bit_exact():
    """Single-token bags return the table row bit for bit (index path, no arithmetic drift)."""
    rng = np.random.default_rng(7)
    V, E, N, L = 5000, 256, 512, 64
    table = cuda(rng.standard_normal((V, E)).astype(np.float32))
    ids = torch.zeros(N, L, dtype=torch.int64, device=DEV)
    rows = torch.as_tensor(rng.integers(1, V, N), device=DEV)
    pos = torch.as_tensor(rng.integers(0, L, N), device=DEV)
    ids[torch.arange(N, device=DEV), pos] = rows
    pooled, _ = ops.bag_mean_forward(table, ids)
    assert torch.equal(pooled, table[rows])


def test_bag_forward_golden(golden):
    g = golden("bag_tiny")
    pooled, denom = ops.bag_mean_forward(cuda(g["table"]), cuda(g["ids"]))
    assert rel(pooled, g["pooled"]) < 1e-6


@pytest.mark.parametrize("E", [64, 128, 256, 48, 512, 1024])
@pytest.mark.parametrize("mode", [_lib.TT_SCATTER_SORTED, _lib.TT_SCATTER_ATOMIC])
def test_bag_backward_vs_oracle(E, mode):
    """Both scatter modes against the oracle; at E >= 256 the sorted mode runs the XCD-sliced
    reduce (4 column slices, V = 1500 leaves a partial row block and padded block groups)."""
    rng = np.random.default_rng(E + 17 * mode)
    V, N, L = 1500, 333, 40
    ids = edge_ids(N, L, V, rng)
    d_pooled = rng.standard_normal((N, E)).astype(np.float32)
    table = cuda(rng.standard_normal((V, E)).astype(np.float32))
    _, denom = ops.bag_mean_forward(table, ids)
    grad = ops.bag_mean_backward(cuda(d_pooled), denom, ids, V, 0, mode)
    ref = O.bag_mean_bwd(d_pooled.astype(np.float64), denom.double().cpu().numpy(), ids.cpu().numpy(), V, 0)
    assert rel(grad, ref) < 1e-5
    assert torch.count_nonzero(grad[0]) == 0


def test_bag_backward_sorted_is_deterministic_and_hot_rows():
    """Char-vocab-like contention (V=34, C1) and a Zipf-hot row: sorted path is bitwise
    reproducible and matches the oracle."""
    rng = np.random.default_rng(3)
    V, N, L, E = 34, 2048, 64, 64
    ids = cuda(rng.integers(0, V, size=(N, L)))
    ids[:, :8] = 5                                   # one very hot row
    d_pooled = cuda(rng.standard_normal((N, E)).astype(np.float32))
    _, denom = ops.bag_mean_forward(cuda(rng.standard_normal((V, E)).astype(np.float32)), ids)
    g1 = ops.bag_mean_backward(d_pooled, denom, ids, V, 0, _lib.TT_SCATTER_SORTED)
    g2 = ops.bag_mean_backward(d_pooled, denom, ids, V, 0, _lib.TT_SCATTER_SORTED)
    assert torch.equal(g1, g2)
    ref = O.bag_mean_bwd(d_pooled.double().cpu().numpy(), denom.double().cpu().numpy(), ids.cpu().numpy(), V, 0)
    assert rel(g1, ref) < 1e-5


@pytest.mark.parametrize("E", [64, 96, 256])
def test_bag_backward_zipf_long_rows_in_pieces(E):
    """Zipf(1.1) ids: rows past 128 tokens are summed in pieces (one wave per piece, partials
    folded in piece order) -- still deterministic and equal to the oracle."""
    rng = np.random.default_rng(12)
    V, N, L = 5000, 6000, 64
    ranks = np.arange(1, V)
    p = ranks ** -1.1
    ids_np = rng.choice(ranks, size=(N, L), p=p / p.sum())
    ids_np[:, 50:] = 0  # padding tail
    ids = cuda(ids_np)
    counts = np.bincount(ids_np[ids_np > 0], minlength=V)
    assert counts.max() > 128 * 256  # the hottest row takes the long-piece length
    d_pooled = cuda(rng.standard_normal((N, E)).astype(np.float32))
    _, denom = ops.bag_mean_forward(cuda(rng.standard_normal((V, E)).astype(np.float32)), ids)
    g1 = ops.bag_mean_backward(d_pooled, denom, ids, V, 0, _lib.TT_SCATTER_SORTED)
    g2 = ops.bag_mean_backward(d_pooled, denom, ids, V, 0, _lib.TT_SCATTER_SORTED)
    assert torch.equal(g1, g2)
    ref = O.bag_mean_bwd(d_pooled.double().cpu().numpy(), denom.double().cpu().numpy(), ids_np, V, 0)
    assert rel(g1, ref) < 1e-5


def test_bag_backward_padding_idx_nonzero():
    rng = np.random.default_rng(4)
    V, N, L, E = 300, 64, 16, 64
    ids = edge_ids(N, L, V, rng)
    ids[:, 2] = 7
    d_pooled = rng.standard_normal((N, E)).astype(np.float32)
    _, denom = ops.bag_mean_forward(cuda(rng.standard_normal((V, E)).astype(np.float32)), ids)
    grad = ops.bag_mean_backward(cuda(d_pooled), denom, ids, V, 7)
    ref = O.bag_mean_bwd(d_pooled.astype(np.float64), denom.double().cpu().numpy(), ids.cpu().numpy(), V, 7)
    assert rel(grad, ref) < 1e-5 and torch.count_nonzero(grad[7]) == 0


def test_bag_backward_empty_batch():
    V, E = 50, 64
    ids = torch.zeros(0, 8, dtype=torch.int64, device=DEV)
    grad = ops.bag_mean_backward(torch.zeros(0, E, device=DEV), torch.zeros(0, device=DEV), ids, V, 0)
    assert grad.shape == (V, E) and torch.count_nonzero(grad) == 0


# ---------------------------------------------------------------------------------------------
# AdamW (dense and fused with the sorted scatter)
def test_adamw_vs_oracle():
    rng = np.random.default_rng(5)
    n = 10007
    p, g = rng.standard_normal(n), rng.standard_normal(n)
    m, v = rng.standard_normal(n) * 0.1, np.abs(rng.standard_normal(n)) * 0.01
    P, G, Mt, Vt = (cuda(x.astype(np.float32)) for x in (p, g, m, v))
    ops.adamw_step(P, G, Mt, Vt, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01, step=7)
    rp, rm, rv = O.adamw(p, g, m, v, 7)
    assert rel(P, rp) < 1e-6 and rel(Mt, rm) < 1e-6 and rel(Vt, rv) < 1e-6


def test_adamw_matches_torch():
    torch.manual_seed(0)
    w1 = torch.randn(513, 77, device=DEV, requires_grad=True)
    w2 = torch.nn.Parameter(w1.detach().clone())
    o1 = torch.optim.AdamW([w1], lr=1e-3)
    o2 = tt.optim.AdamW([w2], lr=1e-3)
    for _ in range(3):
        g = torch.randn_like(w1)
        w1.grad, w2.grad = g.clone(), g.clone()
        o1.step()
        o2.step()
    assert rel(w2, w1) < 1e-6
    assert set(o2.state[w2].keys()) == set(o1.state[w1].keys())


@pytest.mark.parametrize("E", [64, 256, 1024])
def test_fused_table_adamw_equals_dense_path(E):
    rng = np.random.default_rng(6)
    V, N, L = 4000, 300, 32
    ids = edge_ids(N, L, V, rng)
    t0 = rng.standard_normal((V, E)).astype(np.float32)
    d_pooled = cuda(rng.standard_normal((N, E)).astype(np.float32))
    A, B = cuda(t0), cuda(t0)
    mA, vA = torch.zeros_like(A), torch.zeros_like(A)
    mB, vB = torch.zeros_like(B), torch.zeros_like(B)
    _, denom = ops.bag_mean_forward(A, ids)
    for step in (1, 2):
        grad = ops.bag_mean_backward(d_pooled, denom, ids, V, 0)
        ops.adamw_step(A, grad, mA, vA, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01, step=step)
        ops.bag_mean_backward_adamw(d_pooled, denom, ids, B, mB, vB, 0, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8,
                                    weight_decay=0.01, step=step)
    assert torch.equal(A, B) and torch.equal(mA, mB) and torch.equal(vA, vB)


# ---------------------------------------------------------------------------------------------
# normalize + per-sample losses
def test_l2norm_vs_oracle():
    rng = np.random.default_rng(8)
    x = rng.standard_normal((257, 128)).astype(np.float32)
    x[3] = 0.0
    dout = rng.standard_normal(x.shape).astype(np.float32)
    X = cuda(x).requires_grad_(True)
    out = ops.l2_normalize(X)
    out.backward(cuda(dout))
    ro, _ = O.l2norm_fwd(x.astype(np.float64))
    assert rel(out, ro) < 1e-6
    assert rel(X.grad, O.l2norm_bwd(dout.astype(np.float64), x.astype(np.float64))) < 1e-5


def test_triplet_golden(golden):
    g = golden("losses")
    q, p, n = (cuda(g[k]).requires_grad_(True) for k in ("tri_q", "tri_p", "tri_n"))
    loss = tt.losses.contrastive_triplet_loss(q, p, n, margin=float(g["tri_margin"]))
    loss.backward()
    assert abs(loss.item() - g["tri_loss"]) < 1e-5
    assert rel(q.grad, g["tri_dq"]) < 1e-5 and rel(p.grad, g["tri_dp"]) < 1e-5 and rel(n.grad, g["tri_dn"]) < 1e-5


def test_multiple_negatives_golden(golden):
    g = golden("losses")
    q, p, negs = (cuda(g[k]).requires_grad_(True) for k in ("mn_q", "mn_p", "mn_negs"))
    loss = tt.losses.multiple_negatives_loss(q, p, negs, temperature=float(g["mn_tau"]))
    loss.backward()
    assert abs(loss.item() - g["mn_loss"]) < 1e-5
    assert rel(q.grad, g["mn_dq"]) < 1e-5 and rel(p.grad, g["mn_dp"]) < 1e-5 and rel(negs.grad, g["mn_dnegs"]) < 1e-5


@pytest.mark.parametrize("H,N", [(256, 1), (256, 4), (256, 7), (256, 15), (256, 16), (128, 4)])
def test_multiple_negatives_vs_oracle(H, N):
    """multiple_negatives_loss against the fp64 oracle: the H = 256 float4 paths (N <= 4 and
    N <= 15) and the generic kernel (N = 16, H = 128), with an all-zero query and an all-zero
    negative (cosine eps clamp, zero norm gradient)."""
    rng = np.random.default_rng(H * 100 + N)
    B = 300
    q = rng.standard_normal((B, H)).astype(np.float32)
    p = rng.standard_normal((B, H)).astype(np.float32)
    negs = rng.standard_normal((B, N, H)).astype(np.float32)
    q[5] = 0.0
    negs[7, N - 1] = 0.0
    Q, P, Nn = (cuda(x).requires_grad_(True) for x in (q, p, negs))
    loss = tt.losses.multiple_negatives_loss(Q, P, Nn, temperature=0.1)
    loss.backward()
    rl, (rdq, rdp, rdn) = O.multi_neg_fwd_bwd(q.astype(np.float64), p.astype(np.float64), negs.astype(np.float64),
                                              temperature=0.1)
    assert abs(loss.item() - rl) < 1e-5 * max(1.0, abs(rl))
    assert rel(Q.grad, rdq) < 1e-5 and rel(P.grad, rdp) < 1e-5 and rel(Nn.grad, rdn) < 1e-5


def test_multiple_negatives_packed_equals_separate():
    """[q; p; negatives] as consecutive row blocks of one tensor (TwoTower's fused output) take
    MultiNegLossPacked, which writes the three gradients into one tensor: the same loss and the
    same gradients, bit for bit, as three separate tensors."""
    rng = np.random.default_rng(11)
    B, K, H = 300, 4, 256
    x = cuda(rng.standard_normal(((2 + K) * B, H)).astype(np.float32))
    base = x.clone().requires_grad_(True)
    q, p, n = torch.split(base, [B, B, K * B])
    loss = tt.losses.multiple_negatives_loss(q, p, n.view(B, K, H), temperature=0.1)
    assert loss.grad_fn.name().startswith("MultiNegLossPacked")
    loss.backward()
    Q, P, N = (t.detach().clone().requires_grad_(True) for t in torch.split(x, [B, B, K * B]))
    ref = tt.losses.multiple_negatives_loss(Q, P, N.view(B, K, H), temperature=0.1)
    assert not ref.grad_fn.name().startswith("MultiNegLossPacked")
    ref.backward()
    assert torch.equal(loss, ref)
    assert torch.equal(base.grad, torch.cat([Q.grad, P.grad, N.grad]))


# ---------------------------------------------------------------------------------------------
# in-batch scorer
def test_in_batch_golden(golden):
    g = golden("losses")
    for tag in ("ib8", "ib16"):
        q, d = cuda(g[f"{tag}_q"]).requires_grad_(True), cuda(g[f"{tag}_d"]).requires_grad_(True)
        loss = tt.losses.in_batch_sampled_softmax_loss(q, d, temperature=0.1)
        loss.backward()
        assert abs(loss.item() - g[f"{tag}_loss"]) < 1e-5 * max(1, abs(g[f"{tag}_loss"])), tag
        assert rel(q.grad, g[f"{tag}_dq"]) < 1e-5 and rel(d.grad, g[f"{tag}_dd"]) < 1e-5, tag


def _unit(rng, n, H):
    x = rng.standard_normal((n, H))
    return (x / np.linalg.norm(x, axis=1, keepdims=True)).astype(np.float32)


@pytest.mark.parametrize("H", [32, 64, 128, 256])
@pytest.mark.parametrize("B,M,off", [(300, 700, 0), (129, 129, 0), (64, 256, 128), (1000, 2000, 1000)])
@pytest.mark.parametrize("dt", ["fp32", "bf16_split", "bf16"])
def test_in_batch_vs_oracle(H, B, M, off, dt):
    rng = np.random.default_rng(H + B + M)
    q, d = _unit(rng, B, H), _unit(rng, M, H)
    if dt != "fp32":   # the bf16 kernels score bf16-rounded operands: so does the oracle
        q = torch.as_tensor(q).bfloat16().float().numpy()
        d = torch.as_tensor(d).bfloat16().float().numpy()
    Q, D = cuda(q).requires_grad_(True), cuda(d).requires_grad_(True)
    loss = ops.InBatchSoftmaxLoss.apply(Q, D, 10.0, off, dt, None)
    g = 0.7
    loss.backward(torch.tensor(g, device=DEV))
    rl, (rdq, rdd), _ = O.in_batch_fwd_bwd(q.astype(np.float64), d.astype(np.float64), 0.1, g=g, label_off=off)
    tol = {"fp32": 1e-5, "bf16_split": BF16_SPLIT_GRAD_TOL, "bf16": BF16_GRAD_TOL}[dt]
    assert abs(loss.item() - rl) < 1e-5 * max(1.0, abs(rl))
    assert rel(Q.grad, rdq) < tol and rel(D.grad, rdd) < tol


@pytest.mark.parametrize("H", [32, 64, 128, 256])
@pytest.mark.parametrize("B,M,off", [(300, 700, 0), (129, 129, 0), (64, 256, 128), (1000, 2000, 1000),
                                     (1, 64, 0), (320, 330, 10), (448, 900, 0), (2500, 2600, 100)])
def test_in_batch_stored_backward_vs_oracle_and_recompute(H, B, M, off):
    """The default bf16 backward (G from the forward's stored bf16 probabilities,
    score_ddp_kernel) against the float64 oracle on the bf16-rounded operands, and against the
    recompute backward.  The B values give every remainder of the kernel's five-stage rotation
    (query tiles of 64 per split), the exits round 1's wrong-dD race lived on."""
    rng = np.random.default_rng(7 * H + B + M)
    q = torch.as_tensor(_unit(rng, B, H)).bfloat16().float().numpy()
    d = torch.as_tensor(_unit(rng, M, H)).bfloat16().float().numpy()
    g = 0.7
    grads = {}
    prev = ops.get_inbatch_backward()
    try:
        for form in ("stored", "recompute"):
            ops.set_inbatch_backward(form)
            Q, D = cuda(q).requires_grad_(True), cuda(d).requires_grad_(True)
            loss = ops.InBatchSoftmaxLoss.apply(Q, D, 10.0, off, "bf16", None)
            loss.backward(torch.tensor(g, device=DEV))
            grads[form] = (loss.item(), Q.grad.clone(), D.grad.clone())
    finally:
        ops.set_inbatch_backward(prev)
    rl, (rdq, rdd), _ = O.in_batch_fwd_bwd(q.astype(np.float64), d.astype(np.float64), 0.1, g=g, label_off=off)
    loss, dq, dd = grads["stored"]
    assert abs(loss - rl) < 1e-5 * max(1.0, abs(rl))
    assert rel(dq, rdq) < BF16_GRAD_TOL and rel(dd, rdd) < BF16_GRAD_TOL
    # the two backward forms differ only by the rounding of q~ * 2^(shift - lse2) to bf16 (one
    # bf16 rounding, 2^-9, per summed term: largest where few queries contribute)
    assert rel(dd, grads["recompute"][2]) < 4e-3 and torch.equal(dq, grads["recompute"][1])


@pytest.mark.parametrize("H", [32, 64, 128, 256])
@pytest.mark.parametrize("B,M,off", [(300, 700, 0), (129, 129, 0), (64, 256, 128), (1, 64, 0), (320, 330, 10),
                                     (2500, 2600, 100), (768, 800, 16)])
def test_in_batch_fp32_stored_backward_vs_oracle_and_recompute(H, B, M, off):
    """The fp32 stored-probability passes against the float64 oracle at the fp32 bar (1e-5) and
    against the fp32 recompute form (score_f32_kernel, exact f32 MFMA).  H = 64, 128, 256: the
    split-bf16 engines (score_split_fwd_kernel / score_split_ddp_kernel: six bf16 cross products
    per fp32 product, G^T from the forward's fp32 P, the per-query factor folded into three bf16
    planes of the scaled q); H = 32: score_f32_kernel's stored form, whose dq is the recompute
    form's bit for bit (same forward).  B, M off the 32- and 128-row tiles exercise the partial
    blocks; the query tiles per split run 1-3 past the pipelined backward's four-unit loop (B 1 ..
    2500; 768 x 800: three tiles in every split) and 1 past the forward's two-unit loop."""
    rng = np.random.default_rng(11 * H + B + M)
    q, d = _unit(rng, B, H), _unit(rng, M, H)
    g = 0.7
    grads = {}
    prev = ops.get_inbatch_backward()
    try:
        for form in ("stored", "recompute"):
            ops.set_inbatch_backward(form)
            Q, D = cuda(q).requires_grad_(True), cuda(d).requires_grad_(True)
            loss = ops.InBatchSoftmaxLoss.apply(Q, D, 10.0, off, "fp32", None)
            loss.backward(torch.tensor(g, device=DEV))
            grads[form] = (loss.item(), Q.grad.clone(), D.grad.clone())
    finally:
        ops.set_inbatch_backward(prev)
    rl, (rdq, rdd), _ = O.in_batch_fwd_bwd(q.astype(np.float64), d.astype(np.float64), 0.1, g=g, label_off=off)
    loss, dq, dd = grads["stored"]
    assert abs(loss - rl) < 1e-5 * max(1.0, abs(rl))
    assert rel(dq, rdq) < 1e-5 and rel(dd, rdd) < 1e-5
    if H == 32:
        assert torch.equal(dq, grads["recompute"][1])
    else:
        assert rel(dq, grads["recompute"][1]) < 1e-5
    assert rel(dd, grads["recompute"][2]) < 1e-5


def test_in_batch_stored_backward_first_call_of_fresh_process():
    """Round 1's failure showed on the first (cold) call of a process only: run the first bf16
    in-batch forward + backward of a fresh process, with no host sync between the passes, at
    H 32, 64 and 256 (each a first launch of its kernels), against the float64 oracle."""
    import subprocess
    import sys

    code = r"""
import sys, numpy as np, torch
sys.path.insert(0, %r)
from oracle import reference_math as O
from twotower_amd import ops
assert ops.get_inbatch_backward() == "stored"
worst = 0.0
for H in (32, 64, 256):
    rng = np.random.default_rng(H)
    q = rng.standard_normal((300, H)); d = rng.standard_normal((700, H))
    q = torch.as_tensor(q / np.linalg.norm(q, axis=1, keepdims=True)).float().bfloat16().float()
    d = torch.as_tensor(d / np.linalg.norm(d, axis=1, keepdims=True)).float().bfloat16().float()
    Q, D = q.cuda().requires_grad_(True), d.cuda().requires_grad_(True)
    ops.InBatchSoftmaxLoss.apply(Q, D, 10.0, 0, "bf16", None).backward()
    _, (rdq, rdd), _ = O.in_batch_fwd_bwd(q.double().numpy(), d.double().numpy(), 0.1, g=1.0, label_off=0)
    for got, want in ((Q.grad, rdq), (D.grad, rdd)):
        e = float(np.nan_to_num(np.abs(got.double().cpu().numpy() - want).max(), nan=1e9) / np.abs(want).max())
        worst = max(worst, e)
print("WORST", worst)
""" % os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k != "TT_INBATCH_BWD"}
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=100, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    worst = float(r.stdout.split("WORST")[1])
    assert worst < BF16_GRAD_TOL, worst


def _ex_rank(q, d, qb_all, lse2_all, db_all, parts_all, world, rank, inv_tau, dt, g):
    """One rank of the candidate-owner data-parallel loss through the explicit-operand ABI,
    with the 'all-gathered' buffers given (tt_inbatch_prep_rows / _fwd_ex / _bwd_ex)."""
    B, H = q.shape
    M = d.shape[0]
    code = _lib.compute_dtype_code(dt)
    st = torch.cuda.current_stream().cuda_stream
    qb = torch.empty(B + 64, H, dtype=torch.bfloat16, device=DEV)
    qn = torch.empty(B, device=DEV)
    _lib.call("tt_inbatch_prep_rows", q.data_ptr(), B, H, qb.data_ptr(), qn.data_ptr(), None, st)
    db = torch.empty(M + 64, H, dtype=torch.bfloat16, device=DEV)
    ws = torch.empty(_lib.lib().tt_inbatch_ex_ws_size(B, world * M, world * B, M, H, code), dtype=torch.uint8,
                     device=DEV)
    lse, lse2, rows = (torch.empty(B, device=DEV) for _ in range(3))
    loss = torch.empty((), device=DEV)
    dqu, dq, dd = torch.empty(B, H, device=DEV), torch.empty(B, H, device=DEV), torch.empty(M, H, device=DEV)
    _lib.call("tt_inbatch_fwd_ex", qb.data_ptr(), qn.data_ptr(), B, db_all.data_ptr(), parts_all.data_ptr(),
              parts_all.numel(), world * M, H, code, inv_tau, rank * M, 1, lse.data_ptr(), lse2.data_ptr(),
              rows.data_ptr(), loss.data_ptr(), dqu.data_ptr(), ws.data_ptr(), ws.numel(), st)
    _lib.call("tt_inbatch_prep_rows", d.data_ptr(), M, H, db.data_ptr(), None, None, st)
    gl = torch.tensor([g], device=DEV)
    _lib.call("tt_inbatch_bwd_ex", qb_all.data_ptr(), lse2_all.data_ptr(), world * B, rank * B, db.data_ptr(), M, B,
              0, H, code, inv_tau, dqu.data_ptr(), gl.data_ptr(), 1.0 / B, dq.data_ptr(), dd.data_ptr(),
              ws.data_ptr(), ws.numel(), st)
    return loss, lse2, dq, dd


@pytest.mark.parametrize("H,world,B", [(256, 2, 192), (128, 3, 100), (64, 4, 64)])
@pytest.mark.parametrize("dt", ["bf16", "bf16_split"])
def test_in_batch_candidate_owner_ranks_equal_global_batch(H, world, B, dt):
    """Cross-device negatives with candidate-owner gradients, every rank simulated in one
    process: rank r scores its B queries against all world * 2B candidates (labels offset by
    r * 2B) and computes the gradient of its own 2B candidates over all world * B queries.
    Together they must give the single-process loss on the global batch [q_r], [p_r; n_r]
    rank-major, with each rank's loss seeded by g = 1/world and the loss mean per rank."""
    rng = np.random.default_rng(H + world)
    M = 2 * B
    q = [cuda(_unit(rng, B, H)) for _ in range(world)]
    d = [cuda(_unit(rng, M, H)) for _ in range(world)]
    st = torch.cuda.current_stream().cuda_stream
    # the all-gathered buffers
    db_all = torch.zeros(world * M + 64, H, dtype=torch.bfloat16, device=DEV)
    parts_all = torch.empty(world * 512, device=DEV)
    qb_all = torch.zeros(world * B + 64, H, dtype=torch.bfloat16, device=DEV)
    for r in range(world):
        tmp = torch.empty(M + 64, H, dtype=torch.bfloat16, device=DEV)
        _lib.call("tt_inbatch_prep_rows", d[r].data_ptr(), M, H, tmp.data_ptr(), None,
                  parts_all[r * 512:].data_ptr(), st)
        db_all[r * M:(r + 1) * M] = tmp[:M]
        qb_all[r * B:(r + 1) * B] = q[r].bfloat16()
    lse2_all = torch.full((world * B + 64,), float("inf"), device=DEV)
    fwd = []
    for r in range(world):  # forward of every rank first: lse2 is gathered before any backward
        out = _ex_rank(q[r], d[r], qb_all, lse2_all, db_all, parts_all, world, r, 10.0, dt, 1.0 / world)
        fwd.append(out)
    # lse2 of the _ex_rank call above was computed before lse2_all was filled: redo the
    # backward half with the gathered lse2 (forward results are deterministic)
    for r in range(world):
        lse2_all[r * B:(r + 1) * B] = fwd[r][1]
    res = [_ex_rank(q[r], d[r], qb_all, lse2_all, db_all, parts_all, world, r, 10.0, dt, 1.0 / world)
           for r in range(world)]
    # single process on the global batch: queries [q_0..], candidates [d_0..] rank-major,
    # query r*B + i labelled with candidate r*M + i (the local label i of rank r)
    Q = torch.cat(q).requires_grad_(True)
    D = torch.cat(d).requires_grad_(True)
    losses, dQ, dD = [], torch.zeros_like(Q), torch.zeros_like(D)
    prev = ops.set_inbatch_backward("recompute")  # the owner passes recompute G: so does the reference
    for r in range(world):
        qr = Q.detach()[r * B:(r + 1) * B].clone().requires_grad_(True)
        Dr = D.detach().clone().requires_grad_(True)
        lr_ = ops.InBatchSoftmaxLoss.apply(qr, Dr, 10.0, r * M, dt, None)
        lr_.backward(torch.tensor(1.0 / world, device=DEV))
        losses.append(lr_.detach())
        dQ[r * B:(r + 1) * B] += qr.grad
        dD += Dr.grad
    ops.set_inbatch_backward(prev)
    tol_dd = 1e-5
    for r in range(world):
        loss, _, dq, dd = res[r]
        assert abs(loss.item() - losses[r].item()) < 1e-5 * max(1.0, abs(losses[r].item()))
        assert rel(dq, dQ[r * B:(r + 1) * B].double().cpu().numpy()) < 1e-5
        assert rel(dd, dD[r * M:(r + 1) * M].double().cpu().numpy()) < tol_dd


def test_in_batch_three_tensor_form_and_zero_copy_candidates():
    rng = np.random.default_rng(11)
    B, H = 96, 128
    allv = cuda(_unit(rng, 3 * B, H)).requires_grad_(True)
    q, p, n = torch.split(allv, B)
    loss = tt.losses.build("in_batch", temperature=0.1)(q, p, n)
    loss.backward()
    a = allv.detach().double().cpu().numpy()
    rl, (rdq, rdd), _ = O.in_batch_fwd_bwd(a[:B], a[B:], 0.1)
    assert abs(loss.item() - rl) < 1e-5
    assert rel(allv.grad[:B], rdq) < 1e-5 and rel(allv.grad[B:], rdd) < 1e-5


def test_packed_losses_equal_separate_tensors():
    """[q; p; n] in one tensor (TwoTower's fused output) takes the packed kernels; results must
    equal the separate-tensor path exactly (same kernels, same operands)."""
    rng = np.random.default_rng(12)
    B, H = 200, 64
    base = _unit(rng, 3 * B, H)
    for name, kw in (("triplet", {"margin": 0.2}), ("in_batch", {"temperature": 0.05})):
        fn = tt.losses.build(name, **kw)
        packed = cuda(base).requires_grad_(True)
        lp = fn(*torch.split(packed, B))
        lp.backward()
        sep = [cuda(base[i * B:(i + 1) * B]).requires_grad_(True) for i in range(3)]
        ls = fn(*sep)
        ls.backward()
        assert lp.item() == ls.item(), name
        assert torch.equal(packed.grad, torch.cat([t.grad for t in sep])), name
    # views that are not the whole base in order fall back to the separate path
    packed = cuda(base).requires_grad_(True)
    q, p, n = torch.split(packed, B)
    lr_ = tt.losses.build("triplet", margin=0.2)(q, n, p)
    rl, _ = O.triplet_fwd_bwd(base[:B], base[2 * B:], base[B:2 * B], 0.2)
    assert abs(lr_.item() - rl) < 1e-5


@pytest.mark.parametrize("rows,cols", [(1, 4), (255, 24), (257, 128), (24576, 256), (3000, 1028), (0, 64)])
def test_colsum_vs_torch(rows, cols):
    x = torch.randn(rows, cols, device=DEV)
    got = ops.colsum(x)
    want = x.double().sum(0)
    assert torch.allclose(got.double(), want, rtol=1e-5, atol=1e-4 * max(1.0, rows ** 0.5))


def test_relu_bwd_matches_mask():
    for n in (4 * 1000, 1001):
        h = torch.randn(n, device=DEV).clamp_min(0)
        dh = torch.randn(n, device=DEV)
        want = dh * (h > 0)
        ops._lib.call("tt_relu_bwd", dh.data_ptr(), h.data_ptr(), n, _lib.stream_of(dh))
        assert torch.equal(dh, want)


@pytest.mark.parametrize("dt,form", [("fp32", "stored"), ("bf16", "stored"), ("bf16", "recompute"),
                                     ("bf16_split", "stored")])
def test_in_batch_rows_past_the_shift_bound_are_exact(dt, form):
    """F.cross_entropy (losses.py:116) is finite for any logits.  The engine's per-row shift is an
    upper bound c2 |q_i| max|d|; rows whose true max sits more than 100 log2 units below it are
    redone exactly (true row max) instead of underflowing.  tau = 0.005 on unit rows: the 48 queries
    whose positive equals the query reach the bound (engine path), the 48 random ones sit 170-220
    log2 units below it (exact path), in one batch."""
    rng = np.random.default_rng(5)
    H, B, M = 64, 96, 200
    q = rng.standard_normal((B, H))
    d = rng.standard_normal((M, H))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d[:48] = q[:48]
    q, d = q.astype(np.float32), d.astype(np.float32)
    if dt != "fp32":
        q = torch.as_tensor(q).bfloat16().float().numpy()
        d = torch.as_tensor(d).bfloat16().float().numpy()
    prev = ops.set_inbatch_backward(form)
    try:
        Q, D = cuda(q).requires_grad_(True), cuda(d).requires_grad_(True)
        loss = ops.InBatchSoftmaxLoss.apply(Q, D, 200.0, 0, dt, None)   # tau = 0.005
        loss.backward(torch.tensor(1.0, device=DEV))
    finally:
        ops.set_inbatch_backward(prev)
    rl, (rdq, rdd), _ = O.in_batch_fwd_bwd(q.astype(np.float64), d.astype(np.float64), 0.005, g=1.0)
    assert np.isfinite(loss.item()) and torch.isfinite(Q.grad).all() and torch.isfinite(D.grad).all()
    # tau 0.005 puts logits at 200 (x20 the bars' shapes): fp32 rounding of the log2-domain scale c2
    # alone is ~1.7e-5 log2 units there (torch fp32 CPU: 3e-6 on this case, measured 1.3e-5 here)
    tol = {"fp32": 3e-5, "bf16_split": 1e-4, "bf16": 2e-2}[dt]
    print(f"exact-rows {dt}/{form}: loss {abs(loss.item() - rl) / abs(rl):.2e} dq {rel(Q.grad, rdq):.2e} "
          f"dd {rel(D.grad, rdd):.2e}")
    assert abs(loss.item() - rl) < 1e-5 * max(1.0, abs(rl))
    assert rel(Q.grad, rdq) < tol and rel(D.grad, rdd) < tol


# ---------------------------------------------------------------------------------------------
# whole model vs the reference's captured step
def _model_from_fixture(g, V, E, H):
    emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
    model = tt.build_two_tower("mean", emb, hidden_dim=H, tied_weights=True).to(DEV)
    t = model.query_tower
    with torch.no_grad():
        t.embedding.embedding.weight.copy_(cuda(g["table"]))
        t.feed_forward[0].weight.copy_(cuda(g["W1"]))
        t.feed_forward[0].bias.copy_(cuda(g["b1"]))
        t.feed_forward[2].weight.copy_(cuda(g["W2"]))
        t.feed_forward[2].bias.copy_(cuda(g["b2"]))
    return model


@pytest.mark.parametrize("optimizer", ["torch", "tt", "tt_fused"])
def test_c1_step_matches_reference(golden, optimizer):
    g = golden("c1_step")
    V = int(g["V"])
    model = _model_from_fixture(g, V, 64, 128)
    t = model.query_tower
    if optimizer == "torch":
        opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    else:
        opt = tt.optim.AdamW(model.parameters(), lr=1e-3, fused_tables=optimizer == "tt_fused", tables=[t.embedding])
    loss_fn = tt.losses.build("triplet", margin=0.2)
    q, p, n = cuda(g["q"]), cuda(g["p"]), cuda(g["n"])
    qv, pv, nv = model(q, p, n)
    loss = loss_fn(qv, pv, nv)
    opt.zero_grad()
    loss.backward()
    assert abs(loss.item() - g["loss"]) < 1e-5
    assert rel(qv, g["qv"]) < 1e-5 and rel(nv, g["nv"]) < 1e-5
    if optimizer != "tt_fused":
        assert rel(t.embedding.embedding.weight.grad, g["g_table"]) < 1e-5
        assert rel(t.feed_forward[0].weight.grad, g["g_W1"]) < 1e-5
    opt.step()
    assert rel(t.embedding.embedding.weight, g["after_table"]) < 1e-5
    assert rel(t.feed_forward[2].weight, g["after_W2"]) < 1e-5


def test_trajectory_matches_reference(golden):
    g = golden("trajectory")
    model = _model_from_fixture(g, g["table"].shape[0], g["table"].shape[1], g["W1"].shape[0])
    t = model.query_tower
    opt = tt.optim.AdamW(model.parameters(), lr=float(g["lr"]), fused_tables=True, tables=[t.embedding])
    step = tt.TrainStep(model, tt.losses.build("triplet", margin=0.2), opt)
    for s in range(3):
        loss = step(cuda(g[f"q{s}"]), cuda(g[f"p{s}"]), cuda(g[f"n{s}"]))
        assert abs(loss.item() - g[f"loss{s}"]) < 1e-5
        assert rel(t.embedding.embedding.weight, g[f"step{s}_table"]) < 1e-5
        assert rel(t.feed_forward[0].weight, g[f"step{s}_W1"]) < 1e-5


# ---------------------------------------------------------------------------------------------
# split (planned) backward, device-resident AdamW scalars, graph-captured step
@pytest.mark.parametrize("E", [64, 256, 48])
def test_planned_backward_equals_one_shot(E):
    rng = np.random.default_rng(21)
    V, N, L = 3001, 300, 40
    ids = edge_ids(N, L, V, rng, torch.int32)
    dp = cuda(rng.standard_normal((N, E)).astype(np.float32))
    den = cuda((rng.integers(1, L, N) + 1e-9).astype(np.float32))
    want = ops.bag_mean_backward(dp, den, ids, V, 0)
    plan = ops.BagPlan(ids, V, E, 0)
    got = ops.bag_mean_backward_planned(dp, den, plan)
    assert torch.equal(got, want)
    # fused AdamW from the plan with device scalars == one-shot fused call with host scalars
    tbl = cuda(rng.standard_normal((V, E)).astype(np.float32))
    m = cuda(rng.standard_normal((V, E)).astype(np.float32) * 0.01)
    v = cuda(np.abs(rng.standard_normal((V, E))).astype(np.float32) * 1e-4)
    t1, m1, v1 = tbl.clone(), m.clone(), v.clone()
    ops.bag_mean_backward_adamw(dp, den, ids, t1, m1, v1, 0, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8,
                                weight_decay=0.01, step=3)
    step = torch.tensor(2.0, device=DEV)
    args = torch.zeros(8, device=DEV)
    ops.adam_prepare([(step, args)], lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01)
    assert step.item() == 3.0
    t2, m2, v2 = tbl.clone(), m.clone(), v.clone()
    ops.bag_mean_backward_adamw_planned(dp, den, ops.BagPlan(ids, V, E, 0), t2, m2, v2, args)
    assert torch.equal(t1, t2) and torch.equal(m1, m2) and torch.equal(v1, v2)


def _plan_out(plan, n):
    """(sorted keys, their sequence indices, seg_start) read out of a BagPlan's buffer."""
    offs = (ctypes.c_int64 * 3)()
    ops.call("tt_bag_plan_layout", plan.nseq, plan.L, plan.V, plan.E, offs)
    torch.cuda.synchronize()
    base = (-plan.buf.data_ptr()) % 256
    raw = plan.buf.cpu().numpy()

    def arr(o, count):
        return raw[base + o: base + o + 4 * count].view(np.int32)

    return arr(offs[0], n).astype(np.int64), arr(offs[1], n).astype(np.int64), arr(offs[2], plan.V + 1)


@pytest.mark.parametrize("case", ["edge-2pass", "one-pass", "c3-uniform", "zipf-hot", "three-pass-i64",
                                  "all-masked", "padding-idx-7"])
def test_plan_sort_equals_stable_sort(case):
    """tt_bag_plan's hand-written LSD counting sort: its sorted keys (tokens only: the masked
    slots are dropped), sequence indices and row
    starts equal the oracle's stable sort (oracle.reference_math.bag_plan), bit for bit, for 1,
    2 and 3 digit passes (V 1000 / 3001, 200000 / 2^23 + 5), ragged and all-padding batches, a
    Zipf-hot id set, int64 ids and a non-zero padding index."""
    rng = np.random.default_rng(31)
    pad = 0
    if case == "edge-2pass":
        V, ids = 3001, edge_ids(300, 40, 3001, rng, torch.int32)
    elif case == "one-pass":
        V, ids = 1000, edge_ids(257, 33, 1000, rng, torch.int64)
    elif case == "c3-uniform":
        V, ids = 200_000, cuda(rng.integers(0, 200_000, size=(2048, 64)), torch.int32)
    elif case == "zipf-hot":
        V = 200_000
        z = np.minimum(rng.zipf(1.2, size=(3000, 64)), V - 1)
        ids = cuda(z, torch.int32)
    elif case == "three-pass-i64":
        V = (1 << 23) + 5
        ids = cuda(rng.integers(0, V + 3, size=(600, 50)), torch.int64)  # ids >= V are masked
    elif case == "all-masked":
        V, ids = 5000, torch.zeros(64, 16, dtype=torch.int32, device=DEV)
    else:
        V, pad = 3001, 7
        ids = edge_ids(300, 40, 3001, rng, torch.int32)
        ids[5:50, 3] = 7
    wk, ws, wst = O.bag_plan(ids.cpu().numpy(), V, pad)
    n = ids.numel()
    plan = ops.BagPlan(ids, V, 64, pad)
    plan.wait()
    for split in (False, True):  # split: the ABI's two halves (tt_bag_plan_part 0, then 1) redo it
        if split:
            plan.buf.zero_()
            for part in (0, 1):
                ops.call("tt_bag_plan_part", plan.ids.data_ptr(), _lib.ids_dtype_code(plan.ids), plan.nseq, plan.L,
                         plan.L, V, 64, plan.pad, plan.buf.data_ptr(), plan.buf.numel(), part,
                         torch.cuda.current_stream().cuda_stream)
        keys, seqs, starts = _plan_out(plan, n)
        # the sort's first pass drops the masked slots (the oracle sorts them last under key V):
        # the tokens' prefix is the whole plan
        nv = int(wst[V])
        assert np.array_equal(keys[:nv], wk[:nv]), split
        assert np.array_equal(seqs[:nv], ws[:nv]), split
        assert np.array_equal(starts, wst), split


@pytest.mark.parametrize("E,denom", [(256, True), (64, True), (48, False), (256, False)])
def test_planned_backward_row_ranges_equal_whole(E, denom):
    """The row-range form the sharded exchange uses (tt_bag_mean_bwd_planned_prepare once, then
    tt_bag_mean_bwd_planned_rows per chunk, in any order and size, hot rows with pieces included)
    writes exactly the rows of the whole planned gradient, bit for bit; denom None: pre-divided."""
    rng = np.random.default_rng(24)
    V, N, L = 3001, 500, 300  # L 300: rows with > 128 tokens take the piece path
    ids = edge_ids(N, L, V, rng, torch.int32)
    ids[:40, :200] = 17  # a hot row
    dp = cuda(rng.standard_normal((N, E)).astype(np.float32))
    den = cuda((rng.integers(1, L, N) + 1e-9).astype(np.float32)) if denom else None
    plan = ops.BagPlan(ids, V, E, 0)
    want = ops.bag_mean_backward_planned(dp, den, plan)
    ops.bag_mean_backward_planned_prepare(dp, den, plan)
    got = torch.full((V, E), float("nan"), device=DEV)
    for lo, hi in ((2000, 3001), (0, 17), (17, 18), (18, 1000), (1000, 2000)):
        ops.bag_mean_backward_planned_rows(dp, den, plan, lo, hi, got[lo:hi])
    assert torch.equal(got, want)


def test_planned_backward_empty_batch():
    V, E = 50, 64
    ids = torch.zeros(0, 8, dtype=torch.int32, device=DEV)
    plan = ops.BagPlan(ids, V, E, 0)
    g = ops.bag_mean_backward_planned(torch.zeros(0, E, device=DEV), torch.zeros(0, device=DEV), plan)
    assert torch.equal(g, torch.zeros(V, E, device=DEV))


def test_adamw_multi_matches_host_adamw():
    rng = np.random.default_rng(22)
    shapes = [(256, 256), (256,), (7,), (1000, 3), (5, 5)]
    params = [cuda(rng.standard_normal(s).astype(np.float32)) for s in shapes]
    grads = [cuda(rng.standard_normal(s).astype(np.float32)) for s in shapes]
    a = [torch.nn.Parameter(p.clone()) for p in params]
    b = [torch.nn.Parameter(p.clone()) for p in params]
    oa = tt.optim.AdamW(a, lr=3e-3, weight_decay=0.05)
    ob = tt.optim.AdamW(b, lr=3e-3, weight_decay=0.05, capturable=True)
    ref = torch.optim.AdamW([torch.nn.Parameter(p.clone()) for p in params], lr=3e-3, weight_decay=0.05)
    for _ in range(4):
        for ps, o in ((a, oa), (b, ob), (ref.param_groups[0]["params"], ref)):
            for p, g in zip(ps, grads):
                p.grad = g.clone()
            o.step()
    for x, y, z in zip(a, b, ref.param_groups[0]["params"]):
        assert rel(y, x) < 1e-7
        assert rel(y, z) < 1e-6
    assert ob.state[b[0]]["step"].device.type == "cuda" and ob.state[b[0]]["step"].item() == 4.0


def test_adamw_scalars_ahead_follow_lr_changes_and_state_loads(monkeypatch):
    """Capturable AdamW forms each step's scalars at the previous step's tail (tt_adam_prepare_ex
    increment 1, ahead 1): an lr changed between steps, a parameter skipped for a step and a
    state_dict loaded mid-run still give torch's AdamW trajectory and step counters."""
    monkeypatch.setenv("TT_ADAM_AHEAD", "1")
    rng = np.random.default_rng(23)
    shapes = [(64, 32), (32,), (5, 7)]
    params = [cuda(rng.standard_normal(s).astype(np.float32)) for s in shapes]
    grads = [[cuda(rng.standard_normal(s).astype(np.float32)) for s in shapes] for _ in range(7)]
    ours = [torch.nn.Parameter(p.clone()) for p in params]
    ref = [torch.nn.Parameter(p.clone()) for p in params]
    # a second param group that never has a gradient (frozen): torch does nothing for it, and
    # the capturable step must not fail on it
    frozen_o, frozen_r = (torch.nn.Parameter(cuda(np.ones(6, np.float32))) for _ in range(2))
    oo = tt.optim.AdamW([{"params": ours}, {"params": [frozen_o]}], lr=2e-3, weight_decay=0.05, capturable=True)
    orf = torch.optim.AdamW([{"params": ref}, {"params": [frozen_r]}], lr=2e-3, weight_decay=0.05)
    for k in range(7):
        if k == 3:  # lr schedule step
            for o in (oo, orf):
                o.param_groups[0]["lr"] = 5e-4
        if k == 5:  # round trip through a state_dict (fresh optimizer, loaded state)
            sd = oo.state_dict()
            oo = tt.optim.AdamW([{"params": ours}, {"params": [frozen_o]}], lr=5e-4, weight_decay=0.05,
                                capturable=True)
            oo.load_state_dict(sd)
        for i, (a, b) in enumerate(zip(ours, ref)):
            skip = k == 4 and i == 1  # no gradient for this parameter this step
            a.grad = None if skip else grads[k][i].clone()
            b.grad = None if skip else grads[k][i].clone()
        oo.step()
        orf.step()
    for a, b in zip(ours, ref):
        assert rel(a, b) < 1e-6
        assert oo.state[a]["step"].item() == float(orf.state[b]["step"])
    assert torch.equal(frozen_o.detach(), frozen_r.detach()) and frozen_o not in oo.state


@pytest.mark.parametrize("graph", [False, True])
def test_trainstep_adam_scalars_ahead_equal_in_front(graph, monkeypatch):
    """TrainStep with the scalars formed a step ahead (default) equals the prepare-in-front order
    (TT_ADAM_AHEAD=0) bit for bit, eager and graph-replayed."""
    V, E, B, L = 4000, 256, 128, 16

    def run():
        torch.manual_seed(12)
        emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
        model = tt.build_two_tower("mean", emb, hidden_dim=E, tied_weights=True).to(DEV)
        opt = tt.optim.AdamW(model.parameters(), lr=1e-3, fused_tables=True, tables=[emb], capturable=True)
        step = tt.TrainStep(model, tt.losses.build("in_batch", temperature=0.1, compute_dtype="bf16"), opt,
                            graph=graph, eager_steps=2)
        losses = [step(*tt.data.synthetic_triplets(B, L, V, seed=90 + k, device=DEV)).clone() for k in range(5)]
        torch.cuda.synchronize()
        return losses, [p.detach().clone() for p in model.parameters()], [opt.state[p]["step"].item()
                                                                          for p in model.parameters()]

    monkeypatch.setenv("TT_ADAM_AHEAD", "1")
    got = run()
    monkeypatch.setenv("TT_ADAM_AHEAD", "0")
    want = run()
    for a, b in zip(got[0], want[0]):
        assert torch.equal(a, b)
    for a, b in zip(got[1], want[1]):
        assert torch.equal(a, b)
    assert got[2] == want[2] == [5.0] * len(got[2])


@pytest.mark.parametrize("loss_name", ["in_batch", "triplet"])
def test_graph_step_equals_eager(loss_name):
    """The graph-replayed step computes exactly what the eager step computes."""
    V, E, B, L = 5000, 64, 96, 20

    def build():
        torch.manual_seed(5)
        emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
        model = tt.build_two_tower("mean", emb, hidden_dim=E, tied_weights=True).to(DEV)
        opt = tt.optim.AdamW(model.parameters(), lr=1e-3, fused_tables=True, tables=[emb], capturable=True)
        kw = {"temperature": 0.1} if loss_name == "in_batch" else {"margin": 0.2}
        return model, opt, tt.losses.build(loss_name, **kw)

    batches = [tt.data.synthetic_triplets(B, L, V, seed=k, device=DEV) for k in range(5)]
    m1, o1, l1 = build()
    s1 = tt.TrainStep(m1, l1, o1)
    m2, o2, l2 = build()
    s2 = tt.TrainStep(m2, l2, o2, graph=True, eager_steps=1)
    for b in batches:
        x1 = s1(*b).clone()
        x2 = s2(*b).clone()
        assert torch.equal(x1, x2)
    assert len(s2._graphs) == 1
    for (n_, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        assert torch.equal(p1, p2), n_


def test_stamped_graph_replay_times_every_op():
    """bench.py's per-op times: a step captured under OpTimer.stamp_capture brackets every C-ABI
    call with two tt_stamp kernels; each replay rewrites them (positive, ordered durations that sum
    to less than the replay's own wall time) and the stamped step computes what an unstamped
    graph step computes."""
    import time
    from twotower_amd import _lib
    V, E, B, L = 5000, 256, 256, 20

    def build():
        torch.manual_seed(9)
        emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
        model = tt.build_two_tower("mean", emb, hidden_dim=E, tied_weights=True).to(DEV)
        opt = tt.optim.AdamW(model.parameters(), lr=1e-3, fused_tables=True, tables=[emb], capturable=True)
        return model, opt, tt.losses.build("in_batch", temperature=0.1, compute_dtype="bf16")

    batches = [tt.data.synthetic_triplets(B, L, V, seed=k, device=DEV) for k in range(4)]
    m1, o1, l1 = build()
    s1 = tt.TrainStep(m1, l1, o1, graph=True, eager_steps=1)
    m2, o2, l2 = build()
    s2 = tt.TrainStep(m2, l2, o2, graph=True, eager_steps=1)
    s1(*batches[0])
    s2(*batches[0])
    with _lib.TIMER.stamp_capture(DEV):
        s2(*batches[1])  # captured with stamps
    s1(*batches[1])
    for b in batches[2:]:
        s1(*b)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s2(*b)
        torch.cuda.synchronize()
        wall_ms = (time.perf_counter() - t0) * 1e3
        times = _lib.TIMER.stamp_summary(DEV)
        assert {"tt_bag_mean_fwd_split", "tt_inbatch_fwd_prepped", "tt_bag_mean_bwd_adamw_planned"} <= set(times)
        flat = [t for v in times.values() for t in v]
        assert all(0.0 < t < wall_ms for t in flat)
    for (n_, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        assert torch.equal(p1, p2), n_


@pytest.mark.parametrize("graph", [False, True])
def test_step_side_stream_wgrad_equals_serial(graph):
    """E = H = 256 (TowerHead): TrainStep computes the head weight gradients on a side stream
    beside the fused table update; the result equals a plain backward + step (all serial)."""
    V, E, B, L = 7000, 256, 160, 24

    def build():
        torch.manual_seed(9)
        emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
        model = tt.build_two_tower("mean", emb, hidden_dim=E, tied_weights=True).to(DEV)
        opt = tt.optim.AdamW(model.parameters(), lr=1e-3, fused_tables=True, tables=[emb], capturable=True)
        return model, opt, tt.losses.build("in_batch", temperature=0.1)

    batches = [tt.data.synthetic_triplets(B, L, V, seed=40 + k, device=DEV) for k in range(4)]
    m1, o1, l1 = build()
    m2, o2, l2 = build()
    s2 = tt.TrainStep(m2, l2, o2, graph=graph, eager_steps=1)
    for b in batches:
        loss1 = l1(*m1(*b))
        o1.zero_grad(set_to_none=True)
        loss1.backward()
        assert not o1._side_grads.events  # no owner active: gradients on the current stream
        o1.step()
        loss2 = s2(*b)
        assert torch.equal(loss1.detach(), loss2)
    assert not o2._side_grads.events and not o2._side_grads.active
    for (n_, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        assert torch.equal(p1, p2), n_


def test_step_side_stream_wgrad_multi_use_head():
    """A head applied three times in one step (towers called one by one): autograd sums its
    weight gradients as they arrive, so they stay on the current stream; still == serial."""
    V, E, B, L = 5000, 256, 96, 16

    class Separate(torch.nn.Module):
        def __init__(self, tower):
            super().__init__()
            self.tower = tower

        def forward(self, q, p, n):
            return self.tower(q), self.tower(p), self.tower(n)

    def build():
        torch.manual_seed(11)
        emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
        model = Separate(tt.encoders.build_tower("mean", emb, hidden_dim=E)).to(DEV)
        opt = tt.optim.AdamW(model.parameters(), lr=1e-3, fused_tables=True, tables=[emb], capturable=True)
        return model, opt, tt.losses.build("triplet", margin=0.2)

    batches = [tt.data.synthetic_triplets(B, L, V, seed=60 + k, device=DEV) for k in range(3)]
    m1, o1, l1 = build()
    m2, o2, l2 = build()
    s2 = tt.TrainStep(m2, l2, o2)
    for b in batches:
        loss1 = l1(*m1(*b))
        o1.zero_grad(set_to_none=True)
        loss1.backward()
        o1.step()
        assert torch.equal(loss1.detach(), s2(*b))
    for (n_, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        assert torch.equal(p1, p2), n_


@pytest.mark.parametrize("tag,H", [("proj", 24), ("noproj", 16)])
def test_avg_pool_tower_golden(golden, tag, H):
    """AveragePoolingTower (encoders.py:84-155), eval mode, against the reference's output and
    parameter gradients (tests/golden/avg_pool.npz)."""
    g = golden("avg_pool")
    emb = tt.embeddings.build("lookup", vocab_size=40, embedding_dim=16)
    tower = tt.build_tower("avg_pool", emb, hidden_dim=H).to(DEV).eval()
    with torch.no_grad():
        for n, p in tower.named_parameters():
            p.copy_(cuda(g[f"{tag}_param_{n}"]))
    y = tower(cuda(g[f"{tag}_ids"]))
    (y * cuda(g[f"{tag}_w"])).sum().backward()
    assert rel(y, g[f"{tag}_out"]) < 1e-5
    for n, p in tower.named_parameters():
        assert rel(p.grad, g[f"{tag}_grad_{n}"]) < 1e-5, n


# ---------------------------------------------------------------------------------------------
# search: cosine scores + top-k (inference/search/two_tower.py:92-103)
@pytest.mark.parametrize("nq,nd,H,k", [(1, 5000, 256, 5), (3, 1000, 128, 64), (17, 3001, 64, 10), (2, 70000, 256, 1000)])
def test_cosine_topk_vs_reference_math(nq, nd, H, k):
    rng = np.random.default_rng(nq + nd)
    q = rng.standard_normal((nq, H)).astype(np.float32)
    d = rng.standard_normal((nd, H)).astype(np.float32)
    d[7] = 0.0                      # zero row: eps clamp
    d[11] = d[10]                   # exact tie: lower index first
    Q, D = cuda(q), cuda(d)
    s = ops.cosine_scores(Q, D)
    ref = torch.nn.functional.cosine_similarity(torch.as_tensor(q).double()[:, None], torch.as_tensor(d).double()[None],
                                                dim=2).numpy()
    assert np.abs(s.cpu().numpy() - ref).max() < 1e-6
    vals, idx = ops.topk_rows(s, k)
    sc = s.cpu().numpy()
    order = np.lexsort((np.arange(nd)[None].repeat(nq, 0), -sc), axis=1)[:, :k]  # desc value, asc index
    assert np.array_equal(idx.cpu().numpy(), order)
    assert np.array_equal(vals.cpu().numpy(), np.take_along_axis(sc, order, 1))


@pytest.mark.parametrize("nq,ncols,k,levels", [(3, 300_000, 100, 50), (2, 1_000_000, 1000, 7), (5, 200_000, 10, 1000000),
                                                (1, 65_536 * 4, 1, 3)])
def test_topk_two_stage_ties_across_chunks(nq, ncols, k, levels):
    """Long rows take the two-stage top-k (tt_topk_rows_ws_size > 0); quantised scores put thousands
    of exact ties on the k-th value across chunk boundaries: the lower columns must win."""
    assert _lib.lib().tt_topk_rows_ws_size(nq, ncols, k) > 0
    g = torch.Generator(device=DEV).manual_seed(ncols + k)
    x = torch.randint(0, levels, (nq, ncols), device=DEV, generator=g).float() / levels
    vals, idx = ops.topk_rows(x, k)
    xs = x.cpu().numpy()
    order = np.lexsort((np.arange(ncols)[None].repeat(nq, 0), -xs), axis=1)[:, :k]
    assert np.array_equal(idx.cpu().numpy(), order)
    assert np.array_equal(vals.cpu().numpy(), np.take_along_axis(xs, order, 1))


def test_topk_two_stage_more_rows_than_grid_y():
    """the two-stage top-k puts rows on grid.y (at most 65,535); a query batch past that
    goes in row blocks.  70,000 rows x 8,192 columns (two-stage at k = 10) against torch.topk (each row
    a permutation: no ties), every row block's first and last rows included."""
    nq, ncols, k = 70_000, 8192, 10
    assert _lib.lib().tt_topk_rows_ws_size(nq, ncols, k) > 0
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.rand(nq, ncols, device=DEV, generator=g).argsort(dim=1).float()  # distinct values per row
    vals, idx = ops.topk_rows(x, k)
    tv, ti = torch.topk(x, k, dim=1)
    assert torch.equal(vals, tv)
    assert torch.equal(idx, ti)


@pytest.mark.parametrize("nq,nd,H", [(40, 2049, 256), (70, 999, 64), (9, 300, 36), (33, 4097, 512), (5, 129, 1024)])
def test_cosine_scores_many_queries_and_widths(nq, nd, H):
    """Query passes (up to 32 per pass, fewer at wide H), partial document tiles, H not a multiple
    of the staged chunk."""
    rng = np.random.default_rng(nq * nd + H)
    q = rng.standard_normal((nq, H)).astype(np.float32)
    d = rng.standard_normal((nd, H)).astype(np.float32)
    s = ops.cosine_scores(cuda(q), cuda(d))
    ref = torch.nn.functional.cosine_similarity(torch.as_tensor(q).double()[:, None], torch.as_tensor(d).double()[None],
                                                dim=2).numpy()
    assert np.abs(s.cpu().numpy() - ref).max() < 1e-6


def test_topk_ties_and_extremes():
    x = torch.tensor([[1.0, 3.0, 3.0, -2.0, 3.0, float("-inf"), 0.0, -0.0]], device=DEV)
    vals, idx = ops.topk_rows(x, 4)
    assert idx.tolist() == [[1, 2, 4, 0]] and vals.tolist() == [[3.0, 3.0, 3.0, 1.0]]
    vals, idx = ops.topk_rows(x, 8)
    assert idx[0, -1].item() == 5


def test_search_matches_reference_fixture(golden):
    """inference/search/two_tower.py:37-115 pinned to the reference itself (tests/golden/search.npz:
    its TwoTowerSearch.index_documents + search on a seeded C1-shaped model): the same weights in
    twotower_amd's towers, the stored ids indexed and searched on the HIP path -- document and query
    embeddings and the top-10 scores within 1e-5, the documents equal where the score is not tied
    (within 1e-6) with its neighbour and the document text is unique; and search() on text returns
    the reference's result dicts."""
    g = golden("search")
    V, E = g["table"].shape
    H = g["W1"].shape[0]
    emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
    model = tt.build_two_tower("mean", emb, hidden_dim=H, tied_weights=True)
    t = model.query_tower
    with torch.no_grad():
        t.embedding.embedding.weight.copy_(torch.as_tensor(g["table"]))
        t.feed_forward[0].weight.copy_(torch.as_tensor(g["W1"]))
        t.feed_forward[0].bias.copy_(torch.as_tensor(g["b1"]))
        t.feed_forward[2].weight.copy_(torch.as_tensor(g["W2"]))
        t.feed_forward[2].bias.copy_(torch.as_tensor(g["b2"]))
    doc_ids = torch.as_tensor(g["doc_ids"], dtype=torch.int32)
    engine = tt.search.TwoTowerSearch(model, device=DEV)
    with _lib.record_calls() as calls:
        engine.index_document_ids(doc_ids)
        scores, idx = engine.search_ids(torch.as_tensor(g["query_ids"]), top_k=g["top_scores"].shape[1])
    assert {"tt_cosine_scores", "tt_topk_rows_ex"} <= set(calls), calls
    assert np.abs(engine.document_embeddings.cpu().numpy() - g["doc_emb"]).max() < 1e-5
    q = engine.encode_queries(torch.as_tensor(g["query_ids"]))
    assert np.abs(q.cpu().numpy() - g["query_emb"]).max() < 1e-5
    sc, ix = scores.cpu().numpy(), idx.cpu().numpy()
    assert np.abs(sc - g["top_scores"]).max() < 1e-5
    ref_s, ref_i = g["top_scores"], g["top_index"]
    gap = np.minimum(np.abs(np.diff(ref_s, axis=1, prepend=np.inf)), np.abs(np.diff(ref_s, axis=1, append=-np.inf)))
    sure = (ref_i >= 0) & (gap > 1e-6)
    assert sure.sum() > 0.8 * sure.size
    assert np.array_equal(ix[sure], ref_i[sure])

    class _FixtureTokenizer:  # the reference tokeniser's two calls, answered from the fixture's ids
        def __init__(self, rows):
            self.rows = {f"text{i}": list(r) for i, r in enumerate(rows)}

        def encode(self, text):
            return self.rows[text]

        def truncate_and_pad(self, seq, max_len):
            return seq[:max_len]

    engine.tokenizer = _FixtureTokenizer(g["query_ids"])
    res = engine.search("text0", top_k=5)
    assert [r["document"] for r in res] == ix[0, :5].tolist()
    assert np.abs(np.array([r["score"] for r in res]) - ref_s[0, :5]).max() < 1e-5


def test_search_index_and_query(tmp_path):
    torch.manual_seed(0)
    V, E = 500, 64
    emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
    model = tt.build_two_tower("mean", emb, hidden_dim=E, tied_weights=True).to(DEV)
    docs = torch.randint(1, V, (300, 16), device=DEV, dtype=torch.int32)
    engine = tt.search.TwoTowerSearch(model, device=DEV)
    engine.index_document_ids(docs)
    qids = docs[[5, 42]].clone()
    scores, idx = engine.search_ids(qids, top_k=3)
    assert idx[:, 0].tolist() == [5, 42]          # a document is its own nearest neighbour (tied towers)
    assert torch.allclose(scores[:, 0], torch.ones(2, device=DEV), atol=1e-5)
    with torch.no_grad():
        ref = torch.nn.functional.cosine_similarity(model.query_tower(qids.long())[:, None],
                                                    engine.document_embeddings[None], dim=2)
    assert torch.allclose(torch.topk(ref, 3).values, scores, atol=1e-5)
    engine.save_index(str(tmp_path / "idx.pt"))
    e2 = tt.search.TwoTowerSearch(model, device=DEV)
    e2.load_index(str(tmp_path / "idx.pt"))
    assert torch.equal(e2.document_embeddings, engine.document_embeddings)


# ---------------------------------------------------------------------------------------------
# device-resident feeder (TripletDataset + DataLoader collate)
class _FakeTripletDataset(torch.utils.data.Dataset):
    """Shaped like the reference's TripletDataset: __getitem__ -> three int64 (L,) tensors."""

    def __init__(self, n, L, V, seed):
        g = torch.Generator().manual_seed(seed)
        self.data = [tuple(torch.randint(0, V, (L,), generator=g) for _ in range(3)) for _ in range(n)]

    def __len__(self):
        return len(self.data)

    def __getitem__(self, i):
        return self.data[i]


def test_device_feeder_matches_dataloader_collate():
    ds = _FakeTripletDataset(103, 12, 500, seed=0)
    store = tt.data.DeviceTripletStore.from_dataset(ds, DEV)
    perm = torch.randperm(len(ds), generator=torch.Generator().manual_seed(3))
    loader = torch.utils.data.DataLoader(ds, batch_size=16, sampler=perm.tolist())
    got = list(store.batches(16, order=perm))
    assert len(got) == len(loader)
    for (q, p, n), (rq, rp, rn) in zip(got, loader):
        assert torch.equal(q.cpu().long(), rq) and torch.equal(p.cpu().long(), rp) and torch.equal(n.cpu().long(), rn)
        assert q.dtype == torch.int32 and q._base is p._base  # packed [q; p; n]
    assert not store.bad_index()
    # out-of-range index: padding row + flag, and the next good gather reads clear
    q, p, n = store.gather(torch.tensor([0, 1000], device=DEV))
    assert torch.equal(q[1], torch.zeros_like(q[1])) and store.bad_index()
    store.gather(torch.tensor([0, 1], device=DEV))
    assert not store.bad_index()


@pytest.mark.parametrize("N,L,B", [(1000, 64, 777), (50, 7, 33), (300, 130, 256), (10, 256, 5)])
def test_device_feeder_gather_equals_index_select(N, L, B):
    rows = torch.randint(0, 10_000, (3, N, L), dtype=torch.int32, device=DEV)
    store = tt.data.DeviceTripletStore(rows)
    idx = torch.randint(0, N, (B,), device=DEV)
    q, p, n = store.gather(idx)
    for k, t in enumerate((q, p, n)):
        assert torch.equal(t, rows[k].index_select(0, idx))
    assert not store.bad_index()


@pytest.mark.parametrize("rows,H", [(37, 24), (1000, 256), (5, 1024), (24576, 128), (3000, 200), (7, 2048)])
def test_layernorm_l2_normalize_vs_torch_fp64(rows, H):
    rng = np.random.default_rng(rows + H)
    x = rng.standard_normal((rows, H)).astype(np.float32) * 3 + 1
    x[0] = 2.5  # constant row: var 0
    gm = rng.standard_normal(H).astype(np.float32)
    bt = rng.standard_normal(H).astype(np.float32)
    w = rng.standard_normal((rows, H)).astype(np.float32)
    X, G, Bt = (cuda(a).requires_grad_(True) for a in (x, gm, bt))
    out = ops.layernorm_l2_normalize(X, G, Bt, 1e-5)
    (out * cuda(w)).sum().backward()
    Xr, Gr, Br = (torch.as_tensor(a).double().requires_grad_(True) for a in (x, gm, bt))
    ref = torch.nn.functional.normalize(torch.nn.functional.layer_norm(Xr, (H,), Gr, Br, 1e-5), dim=-1)
    (ref * torch.as_tensor(w).double()).sum().backward()
    assert rel(out, ref) < 1e-5
    assert rel(X.grad, Xr.grad) < 1e-5 and rel(G.grad, Gr.grad) < 1e-5 and rel(Bt.grad, Br.grad) < 1e-5


# ---------------------------------------------------------------------------------------------
# tower head on split-bf16 MFMA GEMMs (H in {128, 256}, E in {64, 128, 256})
@pytest.mark.parametrize("rows,E,H", [(1, 256, 256), (130, 256, 256), (24576, 256, 256), (288, 256, 256),
                                      (1, 128, 128), (130, 128, 128), (12288, 128, 128), (300, 128, 128),
                                      (1, 64, 128), (64, 64, 128), (130, 64, 128), (4099, 64, 128),
                                      (300, 64, 256), (257, 128, 256), (131, 256, 128)])
def test_tower_head_vs_oracle(rows, E, H):
    """The hand-written head at every width it takes (C3 / C5 d = 256, C2 d = 128, C1's char tower
    E = 64 -> H = 128, and the mixed widths) against float64."""
    rng = np.random.default_rng(rows + E)
    x = rng.standard_normal((rows, E)).astype(np.float32)
    W1 = (rng.standard_normal((H, E)) / 16).astype(np.float32)
    b1 = (rng.standard_normal(H) / 16).astype(np.float32)
    W2 = (rng.standard_normal((H, H)) / 16).astype(np.float32)
    b2 = (rng.standard_normal(H) / 16).astype(np.float32)
    g = rng.standard_normal((rows, H)).astype(np.float32)
    X, A, a, B, b = (cuda(t).requires_grad_(True) for t in (x, W1, b1, W2, b2))
    out = ops.tower_head(X, A, a, B, b)
    (out * cuda(g)).sum().backward()
    xd = x.astype(np.float64)
    y, cache = O.ff_fwd(xd, W1.astype(np.float64), b1.astype(np.float64), W2.astype(np.float64), b2.astype(np.float64))
    ref, _ = O.l2norm_fwd(y)
    assert rel(out, ref) < 1e-5
    dy = O.l2norm_bwd(g.astype(np.float64), y)
    # a pre-activation within 1e-5 of max|h| of zero may take either ReLU branch in any fp32
    # evaluation (6.3 M of them at 24576 x 256 hold a few at ~1e-7): the float64 backward takes the
    # HIP forward's branch there (its epilogue's h > 0), as tests/_step_parity.py does
    pooled, h_pre, _ = cache
    tie = np.abs(h_pre) < 1e-5 * np.abs(h_pre).max()
    if tie.any():
        mask = torch.empty(_lib.lib().tt_head_relu_mask_bytes(rows) // 4, dtype=torch.int32, device=DEV)
        hip_pos = (ops._head_gemm(X.detach(), ops._planes(A.detach(), False), 0, bias=a.detach(), mask=mask, N=H)
                   > 0).cpu().numpy()
        h_pre = np.where(tie, np.where(hip_pos, 1e-300, -1e-300), h_pre)
        cache = (pooled, h_pre, np.maximum(h_pre, 0.0))
    dpooled, grads = O.ff_bwd(dy, cache, W1.astype(np.float64), W2.astype(np.float64))
    assert rel(X.grad, dpooled) < 1e-5
    for t, k in ((A, "W1"), (a, "b1"), (B, "W2"), (b, "b2")):
        assert rel(t.grad, grads[k]) < 1e-5, k


@pytest.mark.gpu
@pytest.mark.parametrize("rows", [1, 45, 1000])
def test_head_relu_mask_bits(rows):
    """The forward's ReLU bitmask is exactly (h > 0): decoded with its tile-private layout (word
    ((r // 32) * 4 + n // 64) * 64 + lane, lane = n % 32 + 32 hh, bit 16 ((n // 32) % 2) + v, for
    r % 32 = (v & 3) + 8 (v >> 2) + 4 hh)."""
    rng = np.random.default_rng(7 + rows)
    x = cuda(rng.standard_normal((rows, 256)).astype(np.float32))
    W = cuda((rng.standard_normal((256, 256)) / 16).astype(np.float32))
    b = cuda((rng.standard_normal(256) / 16).astype(np.float32))
    nwords = _lib.lib().tt_head_relu_mask_bytes(rows) // 4
    mask = torch.zeros(nwords, dtype=torch.int32, device="cuda")
    h = ops._head_gemm(x, ops._planes(W, False), 0, bias=b, mask=mask)
    words = mask.cpu().numpy().view(np.uint32)
    r = np.arange(rows)[:, None]
    n = np.arange(256)[None, :]
    rr = r % 32
    hh = (rr >> 2) & 1
    v = (rr & 3) + 4 * (rr >> 3)
    idx = ((r // 32) * 4 + n // 64) * 64 + (n % 32) + 32 * hh
    bits = (words[idx] >> (16 * ((n // 32) % 2) + v)) & 1
    assert np.array_equal(bits.astype(bool), h.cpu().numpy() > 0)


@pytest.mark.gpu
@pytest.mark.parametrize("NG,NX", [(256, 256), (128, 128), (128, 64), (256, 64), (256, 128), (128, 256)])
@pytest.mark.parametrize("rows", [0, 1, 17, 1000, 24576 + 5])
def test_head_wgrad_vs_fp64(rows, NG, NX):
    """dW = G^T X and db = colsum(G) (autograd's Linear weight / bias gradients) vs float64, square
    and rectangular (tt_head_wgrad_ex: the first Linear of a tower with E != H)."""
    rng = np.random.default_rng(11 + rows)
    g = rng.standard_normal((rows, NG)).astype(np.float32)
    x = rng.standard_normal((rows, NX)).astype(np.float32)
    dW, db = ops.head_wgrad(cuda(g), cuda(x))
    if rows == 0:
        assert float(dW.abs().max()) == 0.0 and float(db.abs().max()) == 0.0
        return
    assert rel(dW, g.astype(np.float64).T @ x.astype(np.float64)) < 1e-5
    assert rel(db, g.astype(np.float64).sum(0)) < 1e-5
    dW2, db2 = ops.head_wgrad(cuda(g), cuda(x))
    assert torch.equal(dW, dW2) and torch.equal(db, db2)  # deterministic


@pytest.mark.parametrize("N", [256, 128])
@pytest.mark.parametrize("rows", [0, 1, 200, 24576])
def test_head_wgrad2_vs_fp64(rows, N):
    """Both head weight gradients in one launch (tt_head_wgrad2, slab partials) and their
    fixed-order sums (tt_head_wgrad2_reduce, queued later, here on another stream) vs float64."""
    rng = np.random.default_rng(31 + rows)
    mats = [rng.standard_normal((rows, N)).astype(np.float32) for _ in range(4)]
    g1, x1, g2, x2 = (cuda(m) for m in mats)
    ws = ops.head_wgrad2(g1, x1, g2, x2)
    out = [torch.empty(N, N, device=DEV), torch.empty(N, device=DEV), torch.empty(N, N, device=DEV),
           torch.empty(N, device=DEV)]
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        ops.head_wgrad2_reduce(ws, *out)
    torch.cuda.synchronize()
    dW1, db1, dW2, db2 = out
    if rows == 0:
        assert all(float(t.abs().max()) == 0.0 for t in out)
        return
    m = [a.astype(np.float64) for a in mats]
    assert rel(dW1, m[0].T @ m[1]) < 1e-5 and rel(db1, m[0].sum(0)) < 1e-5
    assert rel(dW2, m[2].T @ m[3]) < 1e-5 and rel(db2, m[2].sum(0)) < 1e-5


def test_c5_shaped_step_at_reference_settings():
    """The bench's C5 step shape (1 positive + 4 negatives per query, multiple_negatives loss,
    E = H = 256 TowerHead) at the reference's AdamW settings (eps 1e-8, weight decay 0.01): the
    HIP gradients against the float64 restatement of the reference step (oracle/cpu_step.py's
    tower, losses.py:47-85) within 1e-5, and the fused table AdamW of a graph-replayed TrainStep
    against torch.optim.AdamW on those gradients, elementwise (tests/_step_parity.py)."""
    import _step_parity

    r = _step_parity.run(3000, 256, 24, 48, "multiple_negatives", "fp32", K=4, grad_tol=1e-5, seed=11, graph=True)
    print(r)


