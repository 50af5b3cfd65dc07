"""Device-resident synthetic (query, doc+, doc-) id batches shaped like the reference's
TripletDataset output (twotower/dataset.py:262-285: three (L,) int64 rows per triplet, padded
with PAD = 0 at the end, tokenisers.py:34,71-83), generated on the GPU so the timed loop is
never host-bound (the reference DataLoader collate caps near 3 batches/s at B = 8192).

MS-MARCO-like lengths: queries U{3..12} tokens, documents U{L/2..L}; ids uniform on [1, V) or
Zipf(s) over the vocabulary.  Seeds 0 (q), 1 (d+), 2 (d-) advanced per batch.
"""
from __future__ import annotations

import torch


def _lengths(gen, B, lo, hi, device):
    return torch.randint(lo, hi + 1, (B,), generator=gen, device=device)


def _ids(gen, B, L, V, lengths, dtype, device, zipf_s=None):
    if zipf_s is None:
        ids = torch.randint(1, V, (B, L), generator=gen, device=device, dtype=torch.int64)
    else:
        ranks = torch.arange(1, V, device=device, dtype=torch.float64)
        probs = ranks.pow(-float(zipf_s))
        ids = torch.multinomial(probs / probs.sum(), B * L, replacement=True, generator=gen).view(B, L) + 1
    pos = torch.arange(L, device=device).unsqueeze(0)
    ids = torch.where(pos < lengths.unsqueeze(1), ids, torch.zeros_like(ids))
    return ids.to(dtype)


def synthetic_triplets(B: int, L: int, V: int, *, seed: int = 0, device="cuda", dtype=torch.int32,
                       query_len=(3, 12), doc_len=None, zipf_s=None):
    """One batch (q, p, n), each (B, L) ids with trailing PAD = 0."""
    doc_len = doc_len or (max(1, L // 2), L)
    gens = []
    for k in range(3):
        g = torch.Generator(device=device)
        g.manual_seed(seed * 3 + k)
        gens.append(g)
    ql = _lengths(gens[0], B, min(query_len[0], L), min(query_len[1], L), device)
    pl = _lengths(gens[1], B, doc_len[0], doc_len[1], device)
    nl = _lengths(gens[2], B, doc_len[0], doc_len[1], device)
    return (_ids(gens[0], B, L, V, ql, dtype, device, zipf_s),
            _ids(gens[1], B, L, V, pl, dtype, device, zipf_s),
            _ids(gens[2], B, L, V, nl, dtype, device, zipf_s))


def tokens_per_triplet(L: int, query_len=(3, 12), doc_len=None) -> float:
    """Expected non-pad tokens per (q, d+, d-) triplet for the generator's length laws."""
    doc_len = doc_len or (max(1, L // 2), L)
    ql = (min(query_len[0], L) + min(query_len[1], L)) / 2
    dl = (doc_len[0] + doc_len[1]) / 2
    return ql + 2 * dl
