"""Capture golden vectors from the REFERENCE implementation (run in the build container only;
/root/reference is not present on the GPU box).  Outputs small .npz fixtures next to this
script; the reference source itself is never copied.

The reference's top-level package does not import here (twotower/__init__.py pulls in wandb
and a huggingface_hub API that no longer exists), so its leaf modules are loaded through a
namespace stub — the same modules its train.py uses:
  twotower/embeddings.py, twotower/encoders.py, twotower/losses.py, twotower/tokenisers.py,
  dataset_factory/synthetic_generators.py (C1 text), torch.optim.AdamW (twotower/train.py:359),
  inference/search/two_tower.py (the search fixture).

    python tests/golden/make_golden.py [/root/reference]
"""
from __future__ import annotations

import importlib
import os
import random
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def load_reference(root: str):
    for pkg in ("twotower", "dataset_factory"):
        m = types.ModuleType(pkg)
        m.__path__ = [os.path.join(root, pkg)]
        sys.modules[pkg] = m
    mods = {n: importlib.import_module(f"twotower.{n}") for n in ("embeddings", "encoders", "losses", "tokenisers")}
    mods["gen"] = importlib.import_module("dataset_factory.synthetic_generators")
    # inference/search/two_tower.py (its package __init__ also imports the GloVe search: skipped)
    for pkg, sub in (("inference", "inference"), ("inference.search", os.path.join("inference", "search"))):
        m = types.ModuleType(pkg)
        m.__path__ = [os.path.join(root, sub)]
        sys.modules[pkg] = m
    mods["search"] = importlib.import_module("inference.search.two_tower")
    return mods


def tied_model_params(model) -> dict:
    t = model.query_tower
    return dict(table=t.embedding.embedding.weight.detach().numpy().copy(),
                W1=t.feed_forward[0].weight.detach().numpy().copy(), b1=t.feed_forward[0].bias.detach().numpy().copy(),
                W2=t.feed_forward[2].weight.detach().numpy().copy(), b2=t.feed_forward[2].bias.detach().numpy().copy())


def tied_model_grads(model) -> dict:
    t = model.query_tower
    return dict(g_table=t.embedding.embedding.weight.grad.numpy().copy(),
                g_W1=t.feed_forward[0].weight.grad.numpy().copy(), g_b1=t.feed_forward[0].bias.grad.numpy().copy(),
                g_W2=t.feed_forward[2].weight.grad.numpy().copy(), g_b2=t.feed_forward[2].bias.grad.numpy().copy())


def case_bag_tiny(R):
    """V=97, E=16, H=24, 8 x 12 ids: an all-pad row, interior zeros, repeats, id V-1."""
    torch.manual_seed(1)
    V, E, H = 97, 16, 24
    emb = R["embeddings"].build("lookup", vocab_size=V, embedding_dim=E)
    tower = R["encoders"].build_tower("mean", emb, hidden_dim=H)
    g = torch.Generator().manual_seed(2)
    ids = torch.randint(1, V, (8, 12), generator=g)
    ids[0, :] = 0                                   # all padding
    ids[1, 5:] = 0                                  # trailing padding
    ids[2, [1, 4, 7]] = 0                           # interior zeros (unknown chars, tokenisers.py:59)
    ids[3, :6] = 7                                  # repeated id
    ids[4, 0] = V - 1                               # last row of the table
    ids[5, 3:] = 0
    pooled_box = {}

    def grab(module, inputs, output):  # returns None: the hook must not replace the output
        pooled_box["pooled"] = inputs[0].detach().clone()

    tower.feed_forward.register_forward_hook(grab)
    out = tower(ids)
    g_out = torch.randn(out.shape, generator=g)
    out.backward(g_out)
    p = {"table": emb.embedding.weight.detach().numpy(), "W1": tower.feed_forward[0].weight.detach().numpy(),
         "b1": tower.feed_forward[0].bias.detach().numpy(), "W2": tower.feed_forward[2].weight.detach().numpy(),
         "b2": tower.feed_forward[2].bias.detach().numpy()}
    return dict(ids=ids.numpy(), g_out=g_out.numpy(), pooled=pooled_box["pooled"].numpy(),
                out=out.detach().numpy(), g_table=emb.embedding.weight.grad.numpy(),
                g_W1=tower.feed_forward[0].weight.grad.numpy(), g_b1=tower.feed_forward[0].bias.grad.numpy(),
                g_W2=tower.feed_forward[2].weight.grad.numpy(), g_b2=tower.feed_forward[2].bias.grad.numpy(),
                **{k: v.copy() for k, v in p.items()})


def _c1_batch(R, n_triplets=64, max_len=64):
    """Real C1 input: synthetic text from the reference generator, char tokeniser, padded."""
    random.seed(0)
    gen = R["gen"]
    triplets = []
    while len(triplets) < n_triplets:
        q, pos = gen.create_positive_pair()
        _, neg = gen.create_negative_pair(q)
        triplets.append((q, pos, neg))
    tok = R["tokenisers"].build("char")
    tok.fit([t for tr in triplets for t in tr])
    enc = lambda s: tok.truncate_and_pad(tok.encode(s), max_len)  # noqa: E731 (dataset.py:243-255)
    q = torch.tensor([enc(t[0]) for t in triplets])
    p = torch.tensor([enc(t[1]) for t in triplets])
    n = torch.tensor([enc(t[2]) for t in triplets])
    return q, p, n, tok.vocab_size


def case_c1_step(R):
    """configs/char_tower.yml: E=64, H=128, tied, triplet m=0.2, AdamW lr 1e-3; one step."""
    q, p, n, V = _c1_batch(R)
    torch.manual_seed(3)
    emb = R["embeddings"].build("lookup", vocab_size=V, embedding_dim=64)
    model = R["encoders"].build_two_tower("mean", emb, hidden_dim=128, tied_weights=True)
    init = tied_model_params(model)
    loss_fn = R["losses"].build("triplet", margin=0.2)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    qv, pv, nv = model(q, p, n)
    loss = loss_fn(qv, pv, nv)
    opt.zero_grad()
    loss.backward()
    grads = tied_model_grads(model)
    opt.step()
    after = {f"after_{k}": v for k, v in tied_model_params(model).items()}
    return dict(q=q.numpy(), p=p.numpy(), n=n.numpy(), V=np.int64(V), loss=np.float64(loss.item()),
                qv=qv.detach().numpy(), pv=pv.detach().numpy(), nv=nv.detach().numpy(),
                **init, **grads, **after)


def case_trajectory(R):
    """Tiny tied model, triplet loss, 3 AdamW steps (pins weight decay on untouched rows)."""
    torch.manual_seed(4)
    V, E, H, B, L = 50, 8, 16, 6, 10
    g = torch.Generator().manual_seed(5)
    batches = []
    for _ in range(3):
        ids = [torch.randint(1, V // 2, (B, L), generator=g) for _ in range(3)]  # rows >= V/2 never touched
        for t in ids:
            t[:, L // 2 + 1:] = 0
        batches.append(ids)
    emb = R["embeddings"].build("lookup", vocab_size=V, embedding_dim=E)
    model = R["encoders"].build_two_tower("mean", emb, hidden_dim=H, tied_weights=True)
    init = tied_model_params(model)
    loss_fn = R["losses"].build("triplet", margin=0.2)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2)
    out = {**init}
    for s, (q, p, n) in enumerate(batches):
        out[f"q{s}"], out[f"p{s}"], out[f"n{s}"] = q.numpy(), p.numpy(), n.numpy()
        qv, pv, nv = model(q, p, n)
        loss = loss_fn(qv, pv, nv)
        opt.zero_grad()
        loss.backward()
        opt.step()
        out[f"loss{s}"] = np.float64(loss.item())
        for k, v in tied_model_params(model).items():
            out[f"step{s}_{k}"] = v
    out["lr"] = np.float64(1e-2)
    return out


def case_losses(R):
    L = R["losses"]
    g = torch.Generator().manual_seed(6)
    out = {}
    # triplet on non-unit vectors (exercises the norms inside the cosine)
    q, p, n = (torch.randn(16, 32, generator=g) * 2 for _ in range(3))
    for t in (q, p, n):
        t.requires_grad_(True)
    loss = L.contrastive_triplet_loss(q, p, n, margin=0.5)
    loss.backward()
    out.update(tri_q=q.detach().numpy(), tri_p=p.detach().numpy(), tri_n=n.detach().numpy(), tri_margin=0.5,
               tri_loss=loss.item(), tri_dq=q.grad.numpy(), tri_dp=p.grad.numpy(), tri_dn=n.grad.numpy())
    # multiple negatives, N = 4 (presets/multi_pos_multi_neg.yml:11)
    q, p = torch.randn(8, 32, generator=g), torch.randn(8, 32, generator=g)
    negs = torch.randn(8, 4, 32, generator=g)
    for t in (q, p, negs):
        t.requires_grad_(True)
    loss = L.multiple_negatives_loss(q, p, negs, temperature=0.1)
    loss.backward()
    out.update(mn_q=q.detach().numpy(), mn_p=p.detach().numpy(), mn_negs=negs.detach().numpy(), mn_tau=0.1,
               mn_loss=loss.item(), mn_dq=q.grad.numpy(), mn_dp=p.grad.numpy(), mn_dnegs=negs.grad.numpy())
    # in-batch softmax: M = B and M = 2B, fp32 inputs and bf16-rounded inputs
    for tag, M, bf in (("ib8", 8, False), ("ib16", 16, False), ("ib16bf", 16, True)):
        q = torch.nn.functional.normalize(torch.randn(8, 32, generator=g), dim=-1)
        d = torch.nn.functional.normalize(torch.randn(M, 32, generator=g), dim=-1)
        if bf:
            q, d = q.bfloat16().float(), d.bfloat16().float()
        q.requires_grad_(True)
        d.requires_grad_(True)
        loss = L.in_batch_sampled_softmax_loss(q, d, temperature=0.1)
        loss.backward()
        out.update({f"{tag}_q": q.detach().numpy(), f"{tag}_d": d.detach().numpy(), f"{tag}_loss": loss.item(),
                    f"{tag}_dq": q.grad.numpy(), f"{tag}_dd": d.grad.numpy()})
    return out


def case_state_dict(R):
    """Parameter names/shapes of the reference models (mean tied/untied, avg_pool with and without
    projection) and the layout of its AdamW state_dict: checkpoint compatibility
    (twotower/utils.py:231-330 saves model.state_dict() / optimizer.state_dict())."""
    import json

    out = {}
    emb = R["embeddings"].build("lookup", vocab_size=50, embedding_dim=16)
    models = {
        "mean_tied": R["encoders"].build_two_tower("mean", emb, hidden_dim=24, tied_weights=True),
        "mean_untied": R["encoders"].build_two_tower("mean", emb, hidden_dim=24, tied_weights=False),
        "avg_proj": R["encoders"].build_two_tower("avg_pool", emb, hidden_dim=24, tied_weights=True),
        "avg_noproj": R["encoders"].build_two_tower("avg_pool", emb, hidden_dim=16, tied_weights=True),
    }
    layout = {k: [[n, list(t.shape)] for n, t in m.state_dict().items()] for k, m in models.items()}
    m = models["mean_tied"]
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
    for prm in m.parameters():
        prm.grad = torch.ones_like(prm)
    opt.step()
    sd = opt.state_dict()
    layout["optimizer"] = {"param_group_keys": sorted(sd["param_groups"][0].keys()),
                           "state_keys": sorted(sd["state"][0].keys()), "n_state": len(sd["state"])}
    out["layout_json"] = np.array(json.dumps(layout))
    return out


def case_avg_pool(R):
    """AveragePoolingTower (encoders.py:84-155) in eval mode (dropout = identity): output and
    parameter gradients of sum(out * w) for a seeded batch, with and without the projection."""
    out = {}
    for tag, H in (("proj", 24), ("noproj", 16)):
        torch.manual_seed(11)
        emb = R["embeddings"].build("lookup", vocab_size=40, embedding_dim=16)
        tower = R["encoders"].build_tower("avg_pool", emb, hidden_dim=H)
        tower.eval()
        g = torch.Generator().manual_seed(12)
        ids = torch.randint(1, 40, (6, 9), generator=g)
        ids[0, :] = 0
        ids[1, 4:] = 0
        ids[2, ::2] = 0
        y = tower(ids)
        w = torch.randn(y.shape, generator=g)
        (y * w).sum().backward()
        out[f"{tag}_ids"] = ids.numpy()
        out[f"{tag}_w"] = w.numpy()
        out[f"{tag}_out"] = y.detach().numpy()
        for n, prm in tower.named_parameters():
            out[f"{tag}_param_{n}"] = prm.detach().numpy()
            out[f"{tag}_grad_{n}"] = prm.grad.numpy()
    return out


def case_search(R):
    """inference/search/two_tower.py:37-115: a seeded C1-shaped tied model (E 64, H 128) and the
    reference's char tokeniser over generator text; TwoTowerSearch.index_documents then .search for
    a few queries (top 10).  Stored: the documents' and queries' padded ids (max_len 64, the
    reference's), the weights, the document embeddings, each query's embedding and its results
    (scores and document indices)."""
    random.seed(5)
    gen = R["gen"]
    docs, queries = [], []
    while len(docs) < 300:
        q, pos = gen.create_positive_pair()
        _, neg = gen.create_negative_pair(q)
        docs += [pos, neg]
        if len(queries) < 6:
            queries.append(q)
    queries.append(docs[17])  # a query that is one of the documents: its own score is the top
    tok = R["tokenisers"].build("char")
    tok.fit(docs + queries)
    torch.manual_seed(21)
    emb = R["embeddings"].build("lookup", vocab_size=tok.vocab_size, embedding_dim=64)
    model = R["encoders"].build_two_tower("mean", emb, hidden_dim=128, tied_weights=True)
    engine = R["search"].TwoTowerSearch(model, tok, device="cpu")
    engine.index_documents(docs)
    enc = lambda t: tok.truncate_and_pad(tok.encode(t), 64)  # noqa: E731 (two_tower.py:56-61, :89-90)
    out = dict(doc_ids=np.array([enc(d) for d in docs], dtype=np.int64),
               query_ids=np.array([enc(q) for q in queries], dtype=np.int64),
               doc_emb=engine.document_embeddings.numpy().copy(), **tied_model_params(model))
    scores, index = [], []
    for q in queries:
        res = engine.search(q, top_k=10)
        scores.append([r["score"] for r in res])
        index.append([docs.index(r["document"]) if docs.count(r["document"]) == 1 else -1 for r in res])
    with torch.no_grad():
        out["query_emb"] = model.query_tower(torch.tensor(out["query_ids"])).numpy()
    out["top_scores"] = np.array(scores, dtype=np.float64)
    out["top_index"] = np.array(index, dtype=np.int64)  # -1: a duplicated document text (index ambiguous)
    return out


CASES = (("bag_tiny", case_bag_tiny), ("c1_step", case_c1_step), ("trajectory", case_trajectory),
         ("losses", case_losses), ("state_dict", case_state_dict), ("avg_pool", case_avg_pool),
         ("search", case_search))


def main():
    root = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else "/root/reference"
    only = [a[2:] for a in sys.argv[1:] if a.startswith("--")]  # e.g. --avg_pool
    torch.set_num_threads(1)
    R = load_reference(root)
    for name, fn in CASES:
        if only and name not in only:
            continue
        data = fn(R)
        data["torch_version"] = np.array(torch.__version__)
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **{k: np.asarray(v) for k, v in data.items()})
        print(f"wrote {path} ({os.path.getsize(path)} bytes)")


if __name__ == "__main__":
    main()
