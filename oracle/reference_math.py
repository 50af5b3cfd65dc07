"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

numpy restatement of the reference's two-tower step, float64 by default.  Each function cites
the reference line it restates (paths relative to k0r1g/two-towers).  Gradients are written
out by hand (no autograd) so the oracle shares no code with torch's kernels.
"""
from __future__ import annotations

import numpy as np

COS_EPS = 1e-8      # F.cosine_similarity default (twotower/losses.py:28-29,74)
NORM_EPS = 1e-12    # F.normalize default (twotower/encoders.py:77)
POOL_EPS = 1e-9     # twotower/encoders.py:72


# ----------------------------------------------------------------------------------------------
# Embedding lookup + masked mean pool: embeddings.py:30,40 and encoders.py:62-72
def bag_mean_fwd(table: np.ndarray, ids: np.ndarray, dtype=np.float64):
    """pooled[s] = sum_{t: ids[s,t] > 0} table[ids[s,t]] / (count + 1e-9); also returns denom."""
    ids = np.asarray(ids, dtype=np.int64)
    mask = (ids > 0)                                          # encoders.py:62
    rows = np.asarray(table, dtype=dtype)[np.where(mask, ids, 0)] * mask[..., None]   # :67
    denom = mask.sum(1).astype(dtype) + dtype(POOL_EPS)
    pooled = rows.sum(1) / denom[:, None]                                               # :72
    return pooled, denom


def bag_mean_bwd(d_pooled: np.ndarray, denom: np.ndarray, ids: np.ndarray, V: int, padding_idx: int | None = 0,
                 dtype=np.float64) -> np.ndarray:
    """Dense table gradient: G[id] += d_pooled[s] / denom[s] per non-pad token (autograd of
    encoders.py:67-72 through nn.Embedding's dense backward, padding row excluded)."""
    ids = np.asarray(ids, dtype=np.int64)
    g_seq = np.asarray(d_pooled, dtype=dtype) / np.asarray(denom, dtype=dtype)[:, None]
    G = np.zeros((V, g_seq.shape[1]), dtype=dtype)
    s_idx, t_idx = np.nonzero(ids > 0)
    tok = ids[s_idx, t_idx]
    np.add.at(G, tok, g_seq[s_idx])
    if padding_idx is not None and 0 <= padding_idx < V:
        G[padding_idx] = 0
    return G


def bag_plan(ids: np.ndarray, V: int, padding_idx: int | None = 0):
    """The grouping bag_mean_bwd's scatter-add sums by: every token (s, t) of a kept id (0 < id < V,
    id != padding_idx; masked tokens take key V) as the pair (id, s), stably sorted by id, and
    seg_start[r] = the first sorted position whose key is >= r (r = 0..V).  Row r's gradient is
    the sum of g_seq[s] over its segment, in ascending s: the sorted form of nn.Embedding's dense
    backward (embeddings.py:30,40 via train.py:138).  Returns (keys, seqs, seg_start)."""
    ids = np.asarray(ids, dtype=np.int64)
    nseq, L = ids.shape
    keep = (ids > 0) & (ids < V)
    if padding_idx is not None:
        keep &= ids != padding_idx
    keys = np.where(keep, ids, V).reshape(-1)
    seqs = np.repeat(np.arange(nseq, dtype=np.int64), L)
    order = np.argsort(keys, kind="stable")
    ks = keys[order]
    return ks, seqs[order], np.searchsorted(ks, np.arange(V + 1), side="left")


# ----------------------------------------------------------------------------------------------
# Tower head: Linear(E,H) - ReLU - Linear(H,H) (encoders.py:38-42), F.normalize (encoders.py:77)
def l2norm_fwd(x: np.ndarray):
    n = np.sqrt((x * x).sum(-1))
    den = np.maximum(n, NORM_EPS)
    return x / den[:, None], n


def l2norm_bwd(dout: np.ndarray, x: np.ndarray):
    n = np.sqrt((x * x).sum(-1))
    den = np.maximum(n, NORM_EPS)
    sx = (dout * x).sum(-1)
    coef = np.where(n >= NORM_EPS, sx / (den * den * np.where(n > 0, n, 1.0)), 0.0)
    return dout / den[:, None] - coef[:, None] * x


def ff_fwd(pooled, W1, b1, W2, b2):
    h_pre = pooled @ W1.T + b1
    h = np.maximum(h_pre, 0.0)
    y = h @ W2.T + b2
    return y, (pooled, h_pre, h)


def ff_bwd(dy, cache, W1, W2):
    pooled, h_pre, h = cache
    dW2 = dy.T @ h
    db2 = dy.sum(0)
    dh = dy @ W2
    dh_pre = dh * (h_pre > 0)
    dW1 = dh_pre.T @ pooled
    db1 = dh_pre.sum(0)
    dpooled = dh_pre @ W1
    return dpooled, dict(W1=dW1, b1=db1, W2=dW2, b2=db2)


def tower_fwd(params: dict, ids: np.ndarray, dtype=np.float64):
    """MeanPoolingTower.forward (encoders.py:50-81)."""
    p = {k: np.asarray(v, dtype=dtype) for k, v in params.items()}
    pooled, denom = bag_mean_fwd(p["table"], ids, dtype)
    y, ff_cache = ff_fwd(pooled, p["W1"], p["b1"], p["W2"], p["b2"])
    out, _ = l2norm_fwd(y)
    return out, (ids, denom, y, ff_cache)


def tower_bwd(params: dict, dout: np.ndarray, cache, dtype=np.float64):
    ids, denom, y, ff_cache = cache
    p = {k: np.asarray(v, dtype=dtype) for k, v in params.items()}
    dy = l2norm_bwd(dout, y)
    dpooled, g = ff_bwd(dy, ff_cache, p["W1"], p["W2"])
    g["table"] = bag_mean_bwd(dpooled, denom, ids, p["table"].shape[0], 0, dtype)
    return g


# ----------------------------------------------------------------------------------------------
# Cosine (ATen cosine_similarity: sum((x1/clamp|x1|)(x2/clamp|x2|)), norm differentiated,
# clamp not) used by losses.py:28-29,74
def cosine(a, b):
    na, nb = np.sqrt((a * a).sum(-1)), np.sqrt((b * b).sum(-1))
    return (a * b).sum(-1) / (np.maximum(na, COS_EPS) * np.maximum(nb, COS_EPS)), na, nb


def cosine_bwd(g, a, b):
    c, na, nb = cosine(a, b)
    nac, nbc = np.maximum(na, COS_EPS), np.maximum(nb, COS_EPS)
    inv = 1.0 / (nac * nbc)
    sa = np.where(na > 0, c / (nac * np.where(na > 0, na, 1.0)), 0.0)
    sb = np.where(nb > 0, c / (nbc * np.where(nb > 0, nb, 1.0)), 0.0)
    da = g[..., None] * (b * inv[..., None] - sa[..., None] * a)
    db = g[..., None] * (a * inv[..., None] - sb[..., None] * b)
    return da, db


def triplet_fwd_bwd(q, p, n, margin=0.2, g=1.0):
    """contrastive_triplet_loss (losses.py:9-44) and its gradients."""
    cp, _, _ = cosine(q, p)
    cn, _, _ = cosine(q, n)
    h = margin - cp + cn
    loss = np.maximum(h, 0.0).mean()
    gate = np.where(h > 0, g / q.shape[0], 0.0)
    dq1, dp = cosine_bwd(-gate, q, p)
    dq2, dn = cosine_bwd(gate, q, n)
    return loss, (dq1 + dq2, dp, dn)


def _logsumexp(z, axis=-1):
    m = z.max(axis, keepdims=True)
    return (m + np.log(np.exp(z - m).sum(axis, keepdims=True))).squeeze(axis)


def multi_neg_fwd_bwd(q, p, negs, temperature=0.1, g=1.0):
    """multiple_negatives_loss (losses.py:47-85): CE over [cos(q,p), cos(q,n_k)] / tau, label 0."""
    if negs.ndim == 2:
        negs = negs[:, None, :]
    B, N, H = negs.shape
    docs = np.concatenate([p[:, None, :], negs], 1)
    qx = np.broadcast_to(q[:, None, :], docs.shape)
    c, _, _ = cosine(qx, docs)
    z = c / temperature
    lse = _logsumexp(z)
    loss = (lse - z[:, 0]).mean()
    P = np.exp(z - lse[:, None])
    dz = (P - np.eye(N + 1)[0][None, :]) * (g / B)
    dq_all, ddocs = cosine_bwd(dz / temperature, qx, docs)
    return loss, (dq_all.sum(1), ddocs[:, 0], ddocs[:, 1:])


def in_batch_fwd_bwd(q, d, temperature=0.1, g=1.0, label_off=0):
    """in_batch_sampled_softmax_loss (losses.py:88-118): CE over q d^T / tau, labels arange(B)."""
    B = q.shape[0]
    z = (q @ d.T) / temperature
    lse = _logsumexp(z)
    labels = np.arange(B) + label_off
    loss = (lse - z[np.arange(B), labels]).mean()
    P = np.exp(z - lse[:, None])
    P[np.arange(B), labels] -= 1.0
    dz = P * (g / B)
    return loss, (dz @ d / temperature, dz.T @ q / temperature), lse


# ----------------------------------------------------------------------------------------------
# torch.optim.AdamW (twotower/train.py:359), defaults betas (0.9, 0.999), eps 1e-8, wd 1e-2
def adamw(p, g, m, v, step, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-2):
    p = p * (1 - lr * weight_decay)
    m = m + (1 - beta1) * (g - m)
    v = v * beta2 + (1 - beta2) * g * g
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    den = np.sqrt(v) / np.sqrt(bc2) + eps
    p = p - (lr / bc1) * (m / den)
    return p, m, v


# ----------------------------------------------------------------------------------------------
# One tied-tower training step (twotower/train.py:120-139) composed from the pieces above.
def tied_step_grads(params: dict, q_ids, p_ids, n_ids, loss: str = "triplet", dtype=np.float64, **kw):
    qo, qc = tower_fwd(params, q_ids, dtype)
    po, pc = tower_fwd(params, p_ids, dtype)
    no, nc = tower_fwd(params, n_ids, dtype)
    if loss == "triplet":
        L, (dq, dp, dn) = triplet_fwd_bwd(qo, po, no, kw.get("margin", 0.2))
    elif loss == "multiple_negatives":
        L, (dq, dp, dn) = multi_neg_fwd_bwd(qo, po, no, kw.get("temperature", 0.1))
        dn = dn.reshape(no.shape)
    elif loss == "in_batch":
        L, (dq, dd), _ = in_batch_fwd_bwd(qo, np.concatenate([po, no]), kw.get("temperature", 0.1))
        dp, dn = dd[: po.shape[0]], dd[po.shape[0]:]
    else:
        raise ValueError(loss)
    grads = None
    for dout, cache in ((dq, qc), (dp, pc), (dn, nc)):
        gi = tower_bwd(params, dout, cache, dtype)
        grads = gi if grads is None else {k: grads[k] + gi[k] for k in grads}
    return L, (qo, po, no), grads
