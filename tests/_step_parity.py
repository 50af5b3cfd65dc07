"""Whole-step parity at the reference's own optimizer settings (torch.optim.AdamW defaults behind
twotower/train.py:359: lr 1e-3, betas (0.9, 0.999), eps 1e-8, weight_decay 0.01), in two checks:

1. gradients: the HIP model's plain autograd path (dense table gradient from the planned bag
   backward, tower-head gradients, the loss) against the float64 restatement of the reference
   step (oracle/cpu_step.py: nn.Embedding + masked mean + Linear-ReLU-Linear + F.normalize and the
   reference loss) on the same weights and batch, every element max-normalised per tensor;
2. the update: one fused TrainStep (tables updated by the planned scatter + AdamW, graph replay)
   against torch.optim.AdamW applied to those HIP gradients, elementwise.

Split this way no eps dodge is needed: with eps = 1e-8 an element whose gradient is within
rounding of zero may flip its ~lr-sized first update between ANY two fp32 summation orders, so
the update is checked on the SAME gradients (where it is a smooth function of them), and the
gradients against float64 directly.

bf16 scorers: the check is factored at the scorer's boundary, because a max-normalised bias or
weight gradient is a sum over ~25k rows that cancels to a few % of its terms, which multiplies any
per-row operand error by that cancellation.  (a) The scorer: the float64 loss on the HIP tower
outputs rounded to bf16 (the operands the scorer multiplies), its operand gradients against the
HIP scorer's (the same loss kernels run on the tower outputs as leaves) at grad_tol, the scorer's
measured bf16 error being ~1.6e-5 (profiles/r02_scorer_error_table.jsonl); (b) the towers: the
HIP scorer's own operand gradients back-propagated through the float64 towers (straight through
the rounding) against the HIP parameter gradients at the fp32 bar, 1e-5.  Together they cover
every step of the gradient.

ReLU ties: a hidden pre-activation within rounding of zero may take the other branch in any fp32
evaluation (ATen's or ours) than in float64, and one flipped element moves its bias gradient by
that sample's whole contribution (a few % of a max-normalised sum over a few hundred rows).  The
float64 tower therefore takes the HIP forward's branch for the elements with |h| below 1e-5 of the
largest |h| (their count is reported; usually 0-3 in 10^5) and float64's own branch elsewhere."""
from __future__ import annotations

import torch

import twotower_amd as tt
from oracle.cpu_step import RefTower

DEV = "cuda"
HP = dict(lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01)  # torch defaults, train.py:359 (wd 0.01)


def _ref_key(k: str) -> str:
    return k.split("query_tower.")[1].replace("embedding.embedding", "embedding")


def _loss64(name: str, q, p, n, K: int):
    """The reference losses in float64 (losses.py:9-44 triplet, :47-85 multiple negatives with
    (B, K, H) negatives, :88-118 in-batch over cat[p, n] as the 3-tensor registry entry)."""
    F = torch.nn.functional
    if name == "triplet":
        return F.relu(0.2 - F.cosine_similarity(q, p, dim=1) + F.cosine_similarity(q, n, dim=1)).mean()
    if name == "in_batch":
        logits = (q @ torch.cat([p, n]).T) / 0.1
        return F.cross_entropy(logits, torch.arange(q.shape[0], device=q.device))
    if name == "multiple_negatives":
        docs = torch.cat([p.unsqueeze(1), n.view(q.shape[0], K, q.shape[1])], 1)
        logits = F.cosine_similarity(q.unsqueeze(1).expand_as(docs), docs, dim=2) / 0.1
        return F.cross_entropy(logits, torch.zeros(q.shape[0], dtype=torch.long, device=q.device))
    raise ValueError(name)


def _hip_loss(name: str, compute_dtype: str, K: int):
    if name == "in_batch":
        return tt.losses.build("in_batch", temperature=0.1, compute_dtype=compute_dtype)
    if name == "multiple_negatives":
        mn = tt.losses.build("multiple_negatives", temperature=0.1)
        return lambda q, p, n: mn(q, p, n.view(q.shape[0], K, q.shape[1]))
    return tt.losses.build(name, margin=0.2)


@torch.no_grad()
def _hip_hidden_positive(model, ids: torch.Tensor) -> torch.Tensor:
    """(rows, H) bool: the HIP forward's ReLU branch (h > 0) for these sequences: the bag kernel's
    pooled rows through the model's own first Linear (the split-bf16 head GEMM with its bias + ReLU
    epilogue at the head widths, the library GEMM of ops.TowerFF otherwise)."""
    from twotower_amd import ops

    ff = model.query_tower.feed_forward
    x, _ = ops.bag_mean_forward(model.query_tower.embedding.embedding.weight, ids)
    if ff[0].out_features in ops.HEAD_WIDTHS and x.shape[1] in ops.EMB_WIDTHS:
        mask = torch.empty(ops._lib.lib().tt_head_relu_mask_bytes(x.shape[0]) // 4, dtype=torch.int32, device=x.device)
        h = ops._head_gemm(x, ops._planes(ff[0].weight, False), 0, bias=ff[0].bias, mask=mask, N=ff[0].out_features)
    else:
        h = torch.relu(torch.addmm(ff[0].bias, x, ff[0].weight.T))
    return h > 0


def _tower64(ref, ids: torch.Tensor, hip_pos: torch.Tensor, ties: list) -> torch.Tensor:
    """RefTower.forward (oracle/cpu_step.py: encoders.py:62-77) in float64 with the ReLU branch of
    the elements within 1e-5 of max|h| of zero taken from the HIP forward (hip_pos)."""
    F = torch.nn.functional
    mask = (ids > 0).double().unsqueeze(-1)
    emb = ref.embedding(ids) * mask
    pooled = emb.sum(1) / (mask.sum(1) + 1e-9)
    lin1, _, lin2 = ref.feed_forward
    hp = lin1(pooled)
    tie = hp.detach().abs() < 1e-5 * hp.detach().abs().max()
    ties[0] += int(tie.sum())
    pos = torch.where(tie, hip_pos, hp.detach() > 0)
    return F.normalize(lin2(hp * pos), dim=-1)


def _rel(a: torch.Tensor, b: torch.Tensor) -> float:
    return float((a.double() - b).abs().max() / b.abs().max().clamp_min(1e-300))


def run(V: int, E: int, L: int, B: int, loss: str, compute_dtype: str = "fp32", K: int = 1, grad_tol: float = 1e-5,
        seed: int = 0, graph: bool = False) -> dict:
    torch.manual_seed(seed)
    emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
    model = tt.build_two_tower("mean", emb, hidden_dim=E, tied_weights=True).to(DEV)
    init = {k: v.detach().clone() for k, v in model.named_parameters()}
    batch = tt.data.synthetic_triplets(B, L, V, seed=seed + 100, device=DEV, negatives=K)
    hip_loss = _hip_loss(loss, compute_dtype, K)

    # 1a. HIP gradients, plain autograd path (dense table gradient)
    q, p, n = model(*batch)
    lh = hip_loss(q, p, n)
    lh.backward()
    torch.cuda.synchronize()
    g_hip = {k: v.grad.detach().clone() for k, v in model.named_parameters()}
    qpn_hip = [t.detach() for t in (q, p, n)]
    loss_hip = float(lh)
    del q, p, n, lh
    model.zero_grad(set_to_none=True)
    g_ops = {}
    if compute_dtype != "fp32":  # the scorer's operand gradients: the same loss kernels on the same
        leaves = [t.clone().requires_grad_(True) for t in qpn_hip]  # tower outputs, as leaves
        hip_loss(*leaves).backward()
        g_ops = {i: t.grad for i, t in enumerate(leaves)}
        del leaves

    # 1b. float64 oracle on the same weights and batch, ReLU ties broken as the HIP forward broke them
    ref = RefTower(V, E, E).double().to(DEV)
    ref.load_state_dict({_ref_key(k): v.double() for k, v in init.items()})
    ids = [t.long() for t in batch]
    hip_pos = [_hip_hidden_positive(model, t) for t in batch]
    ties = [0]
    q64, p64, n64 = (_tower64(ref, t, hp, ties) for t, hp in zip(ids, hip_pos))
    if compute_dtype == "fp32":
        l64 = _loss64(loss, q64, p64, n64, K)
        l64.backward()
        scorer_errs, tower_tol = {}, grad_tol
    else:  # (a) the scorer on its operands: the HIP outputs rounded to bf16
        ops_r = [t.bfloat16().double().requires_grad_(True) for t in qpn_hip]
        l64 = _loss64(loss, *ops_r, K)
        l64.backward()
        scorer_errs = {nm: _rel(g_ops[i], t.grad) for i, (nm, t) in enumerate(zip("qpn", ops_r))}
        # (b) the towers on the HIP scorer's own gradients (straight through the rounding)
        torch.autograd.backward([q64, p64, n64], [g_ops[i].double() for i in range(3)])
        tower_tol = 1e-5
    g64 = {k: ref.state_dict(keep_vars=True)[_ref_key(k)].grad for k in init}
    errs = {k: _rel(g_hip[k], g64[k]) for k in init}
    out = {"loss_hip": loss_hip, "loss_ref": float(l64), "grad_err": errs, "scorer_err": scorer_errs,
           "relu_ties": ties[0]}
    assert abs(loss_hip - float(l64)) < 1e-5 * max(1.0, abs(float(l64))), out
    assert all(e < grad_tol for e in scorer_errs.values()), out
    assert all(e < tower_tol for e in errs.values()), out
    del ref, q64, p64, n64, l64, g64

    # 2. the fused training step at the reference's AdamW settings vs torch.optim.AdamW on the
    #    HIP gradients of 1a (same weights, same batch)
    opt = tt.optim.AdamW(model.parameters(), fused_tables=True, tables=[emb], capturable=True, **HP)
    step = tt.TrainStep(model, hip_loss, opt, graph=graph, eager_steps=1)
    if graph:  # one eager step (lazy set-up), then the weights and the optimizer state back to
        step(*batch)  # their start, in place: the checked step is the captured graph's first replay
        with torch.no_grad():
            for k, v in model.named_parameters():
                v.copy_(init[k])
            for st in opt.state.values():
                for t in st.values():
                    t.zero_()
        opt._ahead.clear()  # the scalars formed ahead belong to step 2: prepare step 1's in front
    loss_step = float(step(*batch))
    torch.cuda.synchronize()
    assert abs(loss_step - loss_hip) < 1e-6 * max(1.0, abs(loss_hip)), (loss_step, loss_hip)
    tw = {k: torch.nn.Parameter(v.clone()) for k, v in init.items()}
    for k, w in tw.items():
        w.grad = g_hip[k].clone()
    topt = torch.optim.AdamW(list(tw.values()), **HP)
    topt.step()
    upd = {}
    for k, v in model.named_parameters():
        got, want = v.detach().double(), tw[k].detach().double()
        # a few ulp of the parameter and 1e-5 of the lr-sized update
        tol = 1e-5 * HP["lr"] + 4 * 2.0 ** -24 * want.abs()
        bad = (got - want).abs() > tol
        nbad = int(bad.sum())
        # only elements whose gradient is within rounding of zero may move differently
        if nbad:
            gb = g_hip[k][bad].abs()
            assert float(gb.max()) < 1e-9 and nbad <= max(2, v.numel() // 1_000_000), (k, nbad, float(gb.max()))
        upd[k] = nbad
    out["update_mismatches"] = upd
    return out
