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
                       query_len=(3, 12), doc_len=None, zipf_s=None, negatives: int = 1):
    """One batch (q, p, n) of ids with trailing PAD = 0: q and p (B, L), n (negatives * B, L)
    with the negatives of query b in rows b * negatives + k (multi_pos_multi_neg shape when
    negatives > 1, viewed as (B, negatives, L) by the multiple_negatives loss)."""
    doc_len = doc_len or (max(1, L // 2), L)
    gens = []
    for k in range(3):
        g = torch.Generator(device=device)
        g.manual_seed(seed * 3 + k)
        gens.append(g)
    ql = _lengths(gens[0], B, min(query_len[0], L), min(query_len[1], L), device)
    pl = _lengths(gens[1], B, doc_len[0], doc_len[1], device)
    nb = B * int(negatives)
    nl = _lengths(gens[2], nb, doc_len[0], doc_len[1], device)
    return (_ids(gens[0], B, L, V, ql, dtype, device, zipf_s),
            _ids(gens[1], B, L, V, pl, dtype, device, zipf_s),
            _ids(gens[2], nb, L, V, nl, dtype, device, zipf_s))


def tokens_per_triplet(L: int, query_len=(3, 12), doc_len=None) -> float:
    """Expected non-pad tokens per (q, d+, d-) triplet for the generator's length laws."""
    doc_len = doc_len or (max(1, L // 2), L)
    ql = (min(query_len[0], L) + min(query_len[1], L)) / 2
    dl = (doc_len[0] + doc_len[1]) / 2
    return ql + 2 * dl


class DeviceTripletStore:
    """Device-resident replacement for the reference's TripletDataset + DataLoader hot loop
    (twotower/dataset.py:262-285 __getitem__, twotower/train.py:411-417 DataLoader(shuffle=True),
    collate = torch.stack per field, then .to(device)).

    Every encoded triplet is uploaded once as int32 rows (q, d+, d- stacked: (3, N, L)); HBM
    holds millions of them (a 64-token triplet is 768 B).  ``batches`` shuffles on the device and
    gathers each batch with the HIP row-gather (tt_gather_rows_i32) into one packed (3B, L)
    buffer, yielded as consecutive (q, p, n) views -- the layout the fused TwoTower forward uses
    in place.  Batch i holds the same triplets, in the same order, as the reference's loader
    given the same index permutation (``order``)."""

    def __init__(self, rows: torch.Tensor):
        if rows.dim() != 3 or rows.shape[0] != 3:
            raise ValueError(f"rows must be (3, N, L), got {tuple(rows.shape)}")
        self.rows = rows.to(torch.int32).contiguous()
        self.n, self.L = rows.shape[1], rows.shape[2]
        self._bad, self._gen = None, 0

    @classmethod
    def from_dataset(cls, dataset, device="cuda") -> "DeviceTripletStore":
        """From a reference TripletDataset: its pre-encoded lists when load_to_memory was set,
        else one pass of __getitem__ (host tokenisation happens once, not per epoch)."""
        enc = [getattr(dataset, a, None) for a in ("encoded_queries", "encoded_positive_docs", "encoded_negative_docs")]
        if all(e is not None and len(e) == len(dataset) for e in enc):
            rows = torch.tensor(enc, dtype=torch.int32)
        else:
            items = [dataset[i] for i in range(len(dataset))]
            rows = torch.stack([torch.stack([torch.as_tensor(it[k], dtype=torch.int32) for it in items])
                                for k in range(3)])
        return cls(rows.to(device))

    def __len__(self) -> int:
        return self.n

    def gather(self, index: torch.Tensor, out: torch.Tensor | None = None) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """(q, p, n) int32 rows of the given triplet indices, packed in one (3B, L) buffer."""
        from . import _lib

        _lib.require_gpu(self.rows, index)
        index = index.to(torch.int64).contiguous()
        B = index.shape[0]
        if out is None:
            out = torch.empty(3 * B, self.L, dtype=torch.int32, device=self.rows.device)
        if self._bad is None or self._bad.device != out.device:
            self._bad = torch.zeros(1, dtype=torch.int32, device=out.device)
        self._gen = self._gen % (2 ** 31 - 2) + 1  # a new tag per call: the flag is never cleared
        if self._gen == 1:
            self._bad.zero_()
        _lib.call("tt_gather_rows_i32_ex", self.rows.data_ptr(), self.L, self.n, self.n * self.L, 3, index.data_ptr(),
                  B, self.L, out.data_ptr(), self.L, B * self.L, self._bad.data_ptr(), self._gen, _lib.stream_of(out))
        return tuple(torch.split(out, B))

    def bad_index(self) -> bool:
        """Whether the last gather met an index outside [0, n) (its rows were written as padding).
        Reads a device flag: a host sync."""
        return self._bad is not None and int(self._bad.item()) == self._gen

    def order(self, seed: int = 0, shuffle: bool = True) -> torch.Tensor:
        if not shuffle:
            return torch.arange(self.n, device=self.rows.device)
        g = torch.Generator(device=self.rows.device)
        g.manual_seed(seed)
        return torch.randperm(self.n, generator=g, device=self.rows.device)

    def batches(self, batch_size: int, shuffle: bool = True, seed: int = 0, drop_last: bool = False,
                order: torch.Tensor | None = None):
        perm = self.order(seed, shuffle) if order is None else order.to(self.rows.device)
        stop = self.n - (self.n % batch_size if drop_last else 0)
        for i in range(0, stop, batch_size):
            yield self.gather(perm[i:i + batch_size])
