"""Hybrid (sparse + dense) retrieval with reciprocal-rank fusion and optional reranking
(SURVEY.md §2.B N5): the NeMo Retriever ``hybrid`` / ``ranked_hybrid`` pipelines
(experimental/fm-asr-streaming-rag/deploy/docker-compose-nemo-retriever.yaml:39-66 — sparse
top-k 100, dense top-k 100, ranker top-k 40) and the knowledge-graph example's
FLAT-IP + SPARSE_INVERTED_INDEX search with ``RRFRanker``
(experimental/knowledge_graph_rag/vectorstore/search.py:51-87).

* sparse: the native BM25 index (``_rt.BM25Index``), kept in sync with the vector store;
* dense: the in-HBM vector index;
* fusion: RRF, score(d) = sum over lists of 1 / (k + rank(d)), k = 60;
* ``ranked_hybrid``: the fused top candidates go through the cross-encoder reranker, and the
  outlier filter of the FM-ASR retriever drops passages far below the best
  (experimental/fm-asr-streaming-rag/chain-server/retriever.py:99,317-322).
"""
from __future__ import annotations

import statistics
from typing import Dict, List, Optional, Sequence, Tuple

from .._native import rt
from ..index.vectorstore import Document, VectorStore


def rrf(rankings: Sequence[Sequence[int]], k: int = 60) -> List[Tuple[int, float]]:
    score: Dict[int, float] = {}
    for lst in rankings:
        for r, d in enumerate(lst):
            score[d] = score.get(d, 0.0) + 1.0 / (k + r + 1)
    return sorted(score.items(), key=lambda x: -x[1])


def drop_outliers(scores: List[float]) -> List[bool]:
    """Keep passages within max(stdev, 0.1*|mean|) of the best score."""
    if len(scores) < 2:
        return [True] * len(scores)
    best = max(scores)
    tol = max(statistics.pstdev(scores), 0.1 * abs(statistics.fmean(scores)))
    return [s >= best - tol for s in scores]


class HybridRetriever:
    def __init__(self, store: VectorStore, reranker=None, sparse_k: int = 100, dense_k: int = 100,
                 ranker_k: int = 40, rrf_k: int = 60):
        self.store = store
        self.reranker = reranker
        self.sparse_k, self.dense_k, self.ranker_k, self.rrf_k = sparse_k, dense_k, ranker_k, rrf_k
        self.bm25 = rt.BM25Index()
        self._synced = 0
        self.sync()

    def sync(self):
        """Index any documents added to the vector store since the last call."""
        for i, t in list(self.store.docs.texts.items()):
            if i >= self._synced:
                self.bm25.add(int(i), t)
        self._synced = self.store.docs._next

    def remove(self, ids):
        for i in ids:
            self.bm25.remove(int(i))

    def search(self, query: str, k: int = 4, pipeline: str = "ranked_hybrid") -> List[Tuple[Document, float]]:
        self.sync()
        dense = self.store.similarity_search_with_score(query, self.dense_k)
        dense_ids = [d.metadata["doc_id"] for d, _ in dense]
        if pipeline == "dense":
            return dense[:k]
        sparse_ids = [d for d, _ in self.bm25.search(query, self.sparse_k) if d in self.store.docs.texts]
        fused = rrf([sparse_ids, dense_ids], self.rrf_k)
        if pipeline == "hybrid" or self.reranker is None:
            out = fused[:k]
            return [(Document(self.store.docs.get(d), dict(self.store.docs.metadata(d), doc_id=d)), s) for d, s in out]
        cands = [d for d, _ in fused[: self.ranker_k]]
        texts = [self.store.docs.get(d) for d in cands]
        ranks = self.reranker.rank(query, texts)
        keep = drop_outliers([r["logit"] for r in ranks])
        out = []
        for r, ok in zip(ranks, keep):
            if not ok:
                continue
            d = cands[r["index"]]
            out.append((Document(texts[r["index"]], dict(self.store.docs.metadata(d), doc_id=d)), float(r["logit"])))
            if len(out) == k:
                break
        return out
