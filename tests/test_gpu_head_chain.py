"""The tower head's fused chains (head_chain.hip: tt_head_fwd_chain, tt_head_bwd_chain) against the
four-launch head (tt_head_gemm epi 0 / 4 / 1 / 2 / 3 / 5) on the same planes, and against float64
(encoders.py:38-42,77): the chains form the same split-bf16 products operand for operand, so h, dh,
dx, y and the normalised rows (staged through LDS into head_normalize_kernel's layout and arithmetic) must
equal the unfused kernels' bit for bit, and everything is held to float64 at 1e-5.  Row counts
cover partial tiles, partial 128-row blocks and more row blocks than workgroups (the ring carried
across blocks)."""
import numpy as np
import pytest
import torch

from twotower_amd import _lib, ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _planes(W, transpose):
    return ops._planes(W, transpose)


def _ref64(x, W1, b1, W2, b2):
    x, W1, b1, W2, b2 = (t.double() for t in (x, W1, b1, W2, b2))
    h = torch.relu(x @ W1.T + b1)
    y = h @ W2.T + b2
    return h, y, y / y.norm(dim=1, keepdim=True).clamp_min(1e-12)


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("E,H,rows", [(256, 256, 24576 + 37), (256, 256, 1000), (128, 128, 12288), (64, 128, 777),
                                      (128, 256, 300), (64, 256, 4096), (256, 128, 520), (256, 256, 40000)])
def test_head_chains_equal_unfused_kernels_and_float64(E, H, rows):
    g = torch.Generator(device=DEV).manual_seed(E * 7 + H + rows)
    x = torch.randn(rows, E, device=DEV, generator=g)
    W1 = torch.randn(H, E, device=DEV, generator=g) / E ** 0.5
    b1 = torch.randn(H, device=DEV, generator=g) * 0.1
    W2 = torch.randn(H, H, device=DEV, generator=g) / H ** 0.5
    b2 = torch.randn(H, device=DEV, generator=g) * 0.1
    p1, p2, p1t, p2t = _planes(W1, False), _planes(W2, False), _planes(W1, True), _planes(W2, True)
    st = _lib.stream_of(x)
    # unfused reference kernels
    mask = torch.empty(_lib.lib().tt_head_relu_mask_bytes(rows) // 4, dtype=torch.int32, device=DEV)
    h_u = ops._head_gemm(x, p1, 0, bias=b1, mask=mask, N=H)
    y_u = ops._head_gemm(h_u, p2, 4, bias=b2)
    n_u = torch.empty(rows, device=DEV)
    o_u = ops._head_gemm(h_u, p2, 1, bias=b2, norms=n_u)
    # forward chain, both epilogues
    bits = torch.empty(_lib.lib().tt_head_chain_bits_bytes(rows, H) // 4, dtype=torch.int32, device=DEV)
    h, y, o = (torch.empty(rows, H, device=DEV) for _ in range(3))
    nrm = torch.empty(rows, device=DEV)
    ops.call("tt_head_fwd_chain", x.data_ptr(), rows, E, E, H, p1.data_ptr(), p2.data_ptr(), b1.data_ptr(),
             b2.data_ptr(), bits.data_ptr(), h.data_ptr(), y.data_ptr(), None, 0, st)
    h2 = torch.empty_like(h)
    ops.call("tt_head_fwd_chain", x.data_ptr(), rows, E, E, H, p1.data_ptr(), p2.data_ptr(), b1.data_ptr(),
             b2.data_ptr(), bits.data_ptr(), h2.data_ptr(), o.data_ptr(), nrm.data_ptr(), 1, st)
    torch.cuda.synchronize()
    assert torch.equal(h, h_u) and torch.equal(h2, h_u)
    assert torch.equal(y, y_u)
    assert torch.equal(o, o_u) and torch.equal(nrm, n_u)  # head_normalize_kernel's arithmetic
    h64, y64, o64 = _ref64(x, W1, b1, W2, b2)
    assert _rel(o, o64) < 1e-5 and _rel(nrm, y64.norm(dim=1)) < 1e-5 and _rel(h, h64) < 1e-5
    # backward chain: dh = (dy W2) relu'(h), dx = dh W1 (and / denominators)
    dy = torch.randn(rows, H, device=DEV, generator=g)
    den = torch.randint(1, 64, (rows,), device=DEV, generator=g).float() + 1e-9
    dh_u = ops._head_gemm(dy, p2t, 2, mask=mask, N=H)
    dx_u = ops._head_gemm(dh_u, p1t, 3, N=E)
    dxd_u = ops._head_gemm(dh_u, p1t, 5, bias=den, N=E)
    dh, dhd = torch.empty(rows, H, device=DEV), torch.empty(rows, H, device=DEV)
    dx, dxd = torch.empty(rows, E, device=DEV), torch.empty(rows, E, device=DEV)
    ops.call("tt_head_bwd_chain", dy.data_ptr(), rows, H, E, H, p2t.data_ptr(), p1t.data_ptr(), bits.data_ptr(), None,
             dh.data_ptr(), dx.data_ptr(), st)
    ops.call("tt_head_bwd_chain", dy.data_ptr(), rows, H, E, H, p2t.data_ptr(), p1t.data_ptr(), bits.data_ptr(),
             den.data_ptr(), dhd.data_ptr(), dxd.data_ptr(), st)
    torch.cuda.synchronize()
    assert torch.equal(dh, dh_u) and torch.equal(dhd, dh_u)
    assert torch.equal(dx, dx_u) and torch.equal(dxd, dxd_u)
    dh64 = (dy.double() @ W2.double()) * (h64 > 0)
    assert _rel(dx, dh64 @ W1.double()) < 1e-5


@pytest.mark.parametrize("E,H", [(256, 256), (64, 128), (128, 128)])
def test_tower_head_chain_equals_four_launch_head(E, H, monkeypatch):
    """ops.TowerHead through autograd, TT_HEAD_CHAIN=1 against the four launches (the default): the output, every
    gradient (weights on the side-stream-free path) and the input gradient."""
    g = torch.Generator(device=DEV).manual_seed(5)
    rows = 3000
    x0 = torch.randn(rows, E, device=DEV, generator=g)
    W1 = (torch.randn(H, E, device=DEV, generator=g) / E ** 0.5)
    b1 = torch.randn(H, device=DEV, generator=g) * 0.1
    W2 = torch.randn(H, H, device=DEV, generator=g) / H ** 0.5
    b2 = torch.randn(H, device=DEV, generator=g) * 0.1
    dout = torch.randn(rows, H, device=DEV, generator=g)
    res = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("TT_HEAD_CHAIN", mode)
        x = x0.clone().requires_grad_(True)
        ps = [t.clone().requires_grad_(True) for t in (W1, b1, W2, b2)]
        out = ops.tower_head(x, *ps)
        out.backward(dout)
        torch.cuda.synchronize()
        res[mode] = [out.detach()] + [t.grad for t in [x] + ps]
    for a, b in zip(res["1"], res["0"]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("E,H", [(64, 128), (256, 128), (128, 256), (64, 256)])
def test_avg_pool_projection_linear_head(E, H):
    """AveragePoolingTower's projection Linear(E, H) on the split-bf16 kernels (ops.LinearHead,
    encoders.py:84-155): output and the x / W / b gradients against float64, and the tower in eval
    mode against the same tower whose projection runs F.linear."""
    import twotower_amd as tt

    g = torch.Generator(device=DEV).manual_seed(E + H)
    rows = 2000
    x = torch.randn(rows, E, device=DEV, generator=g).requires_grad_(True)
    W = (torch.randn(H, E, device=DEV, generator=g) / E ** 0.5).requires_grad_(True)
    b = (torch.randn(H, device=DEV, generator=g) * 0.1).requires_grad_(True)
    dy = torch.randn(rows, H, device=DEV, generator=g)
    y = ops.linear(x, W, b)
    y.backward(dy)
    x64, W64, b64 = (t.detach().double().requires_grad_(True) for t in (x, W, b))
    y64 = x64 @ W64.T + b64
    y64.backward(dy.double())
    assert _rel(y, y64) < 1e-5
    for got, want in ((x.grad, x64.grad), (W.grad, W64.grad), (b.grad, b64.grad)):
        assert _rel(got, want) < 1e-5
    emb = tt.embeddings.build("lookup", vocab_size=500, embedding_dim=E)
    tower = tt.build_tower("avg_pool", emb, hidden_dim=H).to(DEV).eval()
    ids = torch.randint(0, 500, (300, 20), device=DEV, generator=g)
    with ops._lib.record_calls() as calls:
        out = tower(ids)
    assert "tt_head_gemm" in calls
    lin, _, ln = tower.projection
    ref = torch.nn.functional.normalize(ln(lin(emb.pool_mean(ids))), dim=-1)
    assert _rel(out, ref) < 1e-5
