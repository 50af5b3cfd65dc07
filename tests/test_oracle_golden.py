"""Pin the CPU oracle (oracle/reference_math.py) to golden vectors captured from the reference's
own modules (tests/golden/make_golden.py).  Runs without a GPU."""
import numpy as np

from oracle import reference_math as O


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)


def params_of(g, prefix=""):
    return {k: g[prefix + k] for k in ("table", "W1", "b1", "W2", "b2")}


def test_bag_tiny_forward(golden):
    g = golden("bag_tiny")
    pooled, denom = O.bag_mean_fwd(g["table"], g["ids"])
    assert rel(pooled, g["pooled"]) < 1e-6
    assert np.all(pooled[0] == 0)                       # all-pad row pools to 0
    assert denom[0] == 1e-9 and denom[1] == 5 + 1e-9
    out, _ = O.tower_fwd(params_of(g), g["ids"])
    assert rel(out, g["out"]) < 1e-6


def test_bag_tiny_backward(golden):
    g = golden("bag_tiny")
    p = params_of(g)
    out, cache = O.tower_fwd(p, g["ids"])
    grads = O.tower_bwd(p, g["g_out"], cache)
    for k in ("table", "W1", "b1", "W2", "b2"):
        assert rel(grads[k], g["g_" + k]) < 1e-5, k
    assert np.all(grads["table"][0] == 0)               # padding row never receives gradient


def test_bag_plan_groups_the_golden_backward(golden):
    """The plan restatement (stable (row, seq) sort + segment starts): summing g_seq over each
    row's segment, in segment order, gives the golden table gradient of the reference."""
    g = golden("bag_tiny")
    p = params_of(g)
    out, cache = O.tower_fwd(p, g["ids"])
    grads = O.tower_bwd(p, g["g_out"], cache)
    V = g["table"].shape[0]
    keys, seqs, starts = O.bag_plan(g["ids"], V)
    assert np.all(np.diff(keys) >= 0) and starts[0] == 0 and starts[V] == np.sum(keys < V)
    for r in range(V):
        seg = seqs[starts[r]:(starts[r + 1] if r < V else len(keys))]
        assert np.all(np.diff(seg) >= 0) and np.all(keys[starts[r]:starts[r] + len(seg)] == r)
    # the gradient from the plan: d_pooled / denom summed per segment
    ids = np.asarray(g["ids"], np.int64)
    _, denom = O.bag_mean_fwd(g["table"], ids)
    dp = O.bag_mean_bwd(np.eye(ids.shape[0]), denom, ids, V)  # row r: sum over its tokens of e_s / denom
    for r in range(1, V):
        want = np.zeros(ids.shape[0])
        for s_ in seqs[starts[r]:starts[r + 1]]:
            want[s_] += 1.0 / denom[s_]
        np.testing.assert_allclose(dp[r], want)
    assert rel(grads["table"], g["g_table"]) < 1e-5


def test_interior_zero_is_masked():
    """encoders.py:62 masks every id 0, not only trailing ones: [3,0,5,0] == [3,5,0,0]."""
    t = np.random.default_rng(0).standard_normal((8, 4))
    a, _ = O.bag_mean_fwd(t, np.array([[3, 0, 5, 0]]))
    b, _ = O.bag_mean_fwd(t, np.array([[3, 5, 0, 0]]))
    np.testing.assert_allclose(a, b)


def test_c1_step(golden):
    g = golden("c1_step")
    p = params_of(g)
    loss, (qv, pv, nv), grads = O.tied_step_grads(p, g["q"], g["p"], g["n"], "triplet", margin=0.2)
    assert abs(loss - g["loss"]) <= 1e-6 * max(1.0, abs(g["loss"]))
    assert rel(qv, g["qv"]) < 1e-5 and rel(nv, g["nv"]) < 1e-5
    for k in ("table", "W1", "b1", "W2", "b2"):
        assert rel(grads[k], g["g_" + k]) < 1e-4, k
        new, _, _ = O.adamw(p[k].astype(np.float64), grads[k], 0.0, 0.0, 1)
        assert rel(new, g["after_" + k]) < 1e-5, k


def test_trajectory_adamw(golden):
    g = golden("trajectory")
    p = {k: v.astype(np.float64) for k, v in params_of(g).items()}
    m = {k: np.zeros_like(v) for k, v in p.items()}
    v = {k: np.zeros_like(x) for k, x in p.items()}
    for s in range(3):
        loss, _, grads = O.tied_step_grads(p, g[f"q{s}"], g[f"p{s}"], g[f"n{s}"], "triplet", margin=0.2)
        assert abs(loss - g[f"loss{s}"]) < 1e-5
        for k in p:
            p[k], m[k], v[k] = O.adamw(p[k], grads[k], m[k], v[k], s + 1, lr=float(g["lr"]))
            assert rel(p[k], g[f"step{s}_{k}"]) < 1e-5, (s, k)
    # rows never indexed still decay through weight decay every step (dense AdamW)
    V = g["table"].shape[0]
    np.testing.assert_allclose(p["table"][V // 2:], g["table"][V // 2:] * (1 - 1e-2 * 1e-2) ** 3, rtol=1e-6)


def test_triplet(golden):
    g = golden("losses")
    loss, (dq, dp, dn) = O.triplet_fwd_bwd(g["tri_q"], g["tri_p"], g["tri_n"], float(g["tri_margin"]))
    assert abs(loss - g["tri_loss"]) < 1e-6
    assert rel(dq, g["tri_dq"]) < 1e-5 and rel(dp, g["tri_dp"]) < 1e-5 and rel(dn, g["tri_dn"]) < 1e-5


def test_multiple_negatives(golden):
    g = golden("losses")
    loss, (dq, dp, dn) = O.multi_neg_fwd_bwd(g["mn_q"], g["mn_p"], g["mn_negs"], float(g["mn_tau"]))
    assert abs(loss - g["mn_loss"]) < 1e-5
    assert rel(dq, g["mn_dq"]) < 1e-5 and rel(dp, g["mn_dp"]) < 1e-5 and rel(dn, g["mn_dnegs"]) < 1e-5


def test_in_batch(golden):
    g = golden("losses")
    for tag in ("ib8", "ib16", "ib16bf"):
        loss, (dq, dd), _ = O.in_batch_fwd_bwd(g[f"{tag}_q"].astype(np.float64), g[f"{tag}_d"].astype(np.float64), 0.1)
        assert abs(loss - g[f"{tag}_loss"]) < 1e-5 * max(1, abs(g[f"{tag}_loss"])), tag
        assert rel(dq, g[f"{tag}_dq"]) < 1e-5 and rel(dd, g[f"{tag}_dd"]) < 1e-5, tag


def test_search_fixture_pins_oracle(golden):
    """inference/search/two_tower.py (index_documents + search, captured from the reference): the
    oracle's tower over the stored ids gives the reference's document and query embeddings, and its
    cosine + index-ordered top-k the reference's scores and documents (where the text is unique)."""
    g = golden("search")
    p = params_of(g)
    docs, _ = O.tower_fwd(p, g["doc_ids"])
    qs, _ = O.tower_fwd(p, g["query_ids"])
    assert rel(docs, g["doc_emb"]) < 1e-6
    assert rel(qs, g["query_emb"]) < 1e-6
    cos = (qs @ docs.T) / np.maximum(np.linalg.norm(qs, axis=1)[:, None] * np.linalg.norm(docs, axis=1)[None], 1e-8)
    k = g["top_scores"].shape[1]
    order = np.lexsort((np.arange(docs.shape[0])[None].repeat(len(qs), 0), -cos), axis=1)[:, :k]
    assert np.abs(np.take_along_axis(cos, order, 1) - g["top_scores"]).max() < 1e-5
    known = g["top_index"] >= 0
    assert np.array_equal(order[known], g["top_index"][known])
