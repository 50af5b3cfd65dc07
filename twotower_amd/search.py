"""Semantic search with the trained towers (inference/search/two_tower.py:16-157; the scoring loop
of twotower/evaluate.py:159-199) on the HIP path: documents are encoded forward-only by the
document tower (fused bag lookup + head, no autograd), and queries are ranked by cosine
similarity with a fused HBM-streaming score kernel and an exact radix-select top-k
(ops.cosine_scores / ops.topk_rows).

Tokenisation stays the caller's (any object with the reference tokeniser's encode() and
truncate_and_pad(), twotower/tokenisers.py); ``index_document_ids`` / ``search_ids`` take ids.
The index is saved as a torch file (weights_only load) instead of the reference's pickle.
"""
from __future__ import annotations

import logging

import torch

from . import ops

logger = logging.getLogger("twotower_amd.search")


class TwoTowerSearch:
    def __init__(self, model, tokenizer=None, device="cuda", max_len: int = 64, batch_size: int = 8192):
        self.model = model.to(device)
        self.tokenizer = tokenizer
        self.device = device
        self.max_len = max_len
        self.batch_size = batch_size
        self.document_embeddings: torch.Tensor | None = None
        self.documents: list | None = None

    # ---- encoding (forward only) ---------------------------------------------------------
    def _ids(self, texts) -> torch.Tensor:
        if self.tokenizer is None:
            raise ValueError("a tokenizer is needed for text input; pass token ids instead")
        rows = [self.tokenizer.truncate_and_pad(self.tokenizer.encode(t), self.max_len) for t in texts]
        return torch.tensor(rows, dtype=torch.int32, device=self.device)

    @torch.no_grad()
    def encode_documents(self, ids: torch.Tensor) -> torch.Tensor:
        self.model.eval()
        outs = [self.model.document_tower(ids[i:i + self.batch_size].to(self.device))
                for i in range(0, ids.shape[0], self.batch_size)]
        return torch.cat(outs, 0) if len(outs) > 1 else outs[0]

    @torch.no_grad()
    def encode_queries(self, ids: torch.Tensor) -> torch.Tensor:
        self.model.eval()
        return self.model.query_tower(ids.to(self.device))

    # ---- index -------------------------------------------------------------------------
    def index_documents(self, documents: list[str]) -> None:
        self.index_document_ids(self._ids(documents), documents)

    def index_document_ids(self, ids: torch.Tensor, documents: list | None = None) -> None:
        self.document_embeddings = self.encode_documents(ids).contiguous()
        self.documents = list(documents) if documents is not None else list(range(ids.shape[0]))
        logger.info(f"Indexed {len(self.documents)} documents")

    # ---- search ------------------------------------------------------------------------
    def search_ids(self, query_ids: torch.Tensor, top_k: int = 5) -> tuple[torch.Tensor, torch.Tensor]:
        """(nq, k) scores and document indices for a batch of tokenised queries."""
        if self.document_embeddings is None:
            raise ValueError("No documents indexed. Call index_documents() first.")
        q = self.encode_queries(query_ids)
        return ops.cosine_topk(q, self.document_embeddings, min(top_k, self.document_embeddings.shape[0]))

    def search(self, query: str, top_k: int = 5) -> list[dict]:
        scores, idx = self.search_ids(self._ids([query]), top_k)
        return [{"document": self.documents[i], "score": s} for s, i in zip(scores[0].tolist(), idx[0].tolist())]

    def save_index(self, filepath: str) -> None:
        if self.document_embeddings is None or self.documents is None:
            raise ValueError("No index to save. Call index_documents() first.")
        torch.save({"embeddings": self.document_embeddings.cpu(), "documents": self.documents}, filepath)

    def load_index(self, filepath: str) -> None:
        data = torch.load(filepath, map_location="cpu", weights_only=True)
        self.document_embeddings = data["embeddings"].to(self.device).contiguous()
        self.documents = data["documents"]
