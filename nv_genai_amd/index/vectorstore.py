"""LangChain-``VectorStore``-shaped facade over the in-HBM index + docstore: the surface the
reference's chains call (``add_documents``, ``similarity_search*``, ``as_retriever`` with
``similarity_score_threshold``, ``delete``; RetrievalAugmentedGeneration/common/utils.py:211-468,
examples/nvidia_api_catalog/chains.py:117-127), with named collections
(``COLLECTION_NAME`` / ``conv_store``), filename bookkeeping and snapshot persistence.
"""
from __future__ import annotations

import json
import os
import threading
import time
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Dict, Iterable, List, Optional, Sequence, Tuple

import torch

from ..observability.metrics import METRICS
from .docstore import DocStore
from .flat import FlatIndex
from .ivf import IVFFlatIndex


@dataclass
class Document:
    page_content: str
    metadata: Dict[str, Any] = field(default_factory=dict)


def _embed_docs(embedder, texts: Sequence[str]) -> torch.Tensor:
    if hasattr(embedder, "embed_documents_tensor"):
        return embedder.embed_documents_tensor(texts)
    if hasattr(embedder, "embed") and hasattr(embedder, "dim"):
        return embedder.embed(texts, "passage")
    return torch.tensor(embedder.embed_documents(list(texts)), dtype=torch.float32)


def _embed_queries(embedder, texts: Sequence[str]) -> torch.Tensor:
    if hasattr(embedder, "embed_query_tensor"):
        return embedder.embed_query_tensor(texts)
    if hasattr(embedder, "embed") and hasattr(embedder, "dim"):
        return embedder.embed(texts, "query")
    return torch.tensor([embedder.embed_query(t) for t in texts], dtype=torch.float32)


class WhitenedEmbedder:
    """Another embedder's vectors mapped through y = normalise((x - mu) W) on ``device``: the
    synthetic REST corpus's query whitening (``chain_server.utils._fill_synthetic``) for an
    encoder the store reaches over HTTP, where the encoder itself cannot be calibrated. The
    in-process engine applies the same transform inside ``EmbeddingEngine.embed_ids``."""

    def __init__(self, inner, mu: torch.Tensor, W: torch.Tensor, device=None):
        self.inner = inner
        dev = torch.device(device) if device is not None else mu.device
        self.mu, self.W = mu.to(dev), W.to(dev)
        self.dim = int(W.shape[1])

    def _apply(self, x: torch.Tensor) -> torch.Tensor:
        y = (x.to(self.W.device, torch.float32) - self.mu) @ self.W
        return y / y.norm(dim=-1, keepdim=True).clamp_min(1e-12)

    def embed_query_tensor(self, texts: Sequence[str]) -> torch.Tensor:
        return self._apply(_embed_queries(self.inner, texts))

    def embed_documents_tensor(self, texts: Sequence[str]) -> torch.Tensor:
        return self._apply(_embed_docs(self.inner, texts))

    def embed_query(self, text: str) -> List[float]:
        return self.embed_query_tensor([text])[0].tolist()

    def embed_documents(self, texts: Sequence[str]) -> List[List[float]]:
        return self.embed_documents_tensor(texts).tolist()


class _QueryBatcher:
    """Coalesces concurrent similarity searches (one per chain-server request thread) into one
    query-encoder forward and one index scan, on a dedicated HIP stream. A search therefore
    never queues behind the LLM step running on the default stream; the batch waits only on
    the store's last index write (``VectorStore._mark_write``). Requests arriving within
    ``wait_s`` of the first share a batch (up to ``max_batch``)."""

    def __init__(self, store: "VectorStore", device: torch.device, max_batch: int = 64, wait_s: float = 0.002):
        import queue as _queue

        self.store, self.max_batch, self.wait_s = store, max_batch, wait_s
        self.q: "_queue.Queue" = _queue.Queue()
        self._empty = _queue.Empty
        self.stream = torch.cuda.Stream(device) if device.type == "cuda" else None
        self.batches = 0
        self.queries = 0
        self.thread = threading.Thread(target=self._loop, name=f"query-batcher-{store.name}", daemon=True)
        self.thread.start()

    def submit(self, query: str, k: int):
        import concurrent.futures as cf

        fut = cf.Future()
        self.q.put((query, k, fut, time.perf_counter()))
        return fut

    def _loop(self):
        while True:
            batch = [self.q.get()]
            deadline = time.monotonic() + self.wait_s
            while len(batch) < self.max_batch:
                left = deadline - time.monotonic()
                if left <= 0:
                    break
                try:
                    batch.append(self.q.get(timeout=left))
                except self._empty:
                    break
            t0 = time.perf_counter()
            for b in batch:
                METRICS.observe("retrieval_queue_seconds", t0 - b[3])
            METRICS.observe("retrieval_batch_size", len(batch))
            try:
                if self.stream is not None:
                    ev = self.store._write_ev
                    if ev is not None:
                        self.stream.wait_event(ev)
                    with torch.cuda.stream(self.stream):
                        res = self.store.similarity_search_with_score_batch([b[0] for b in batch],
                                                                            max(b[1] for b in batch))
                else:
                    res = self.store.similarity_search_with_score_batch([b[0] for b in batch],
                                                                        max(b[1] for b in batch))
                METRICS.observe("retrieval_exec_seconds", time.perf_counter() - t0)
                for (_, k, fut, _), r in zip(batch, res):
                    fut.set_result(r[:k])
                self.batches += 1
                self.queries += len(batch)
            except BaseException as e:  # noqa: BLE001 - delivered to every waiting request
                for _, _, fut, _ in batch:
                    if not fut.done():
                        fut.set_exception(e)


class VectorStore:
    def __init__(self, embedder, dim: int, index_type: str = "flat", metric: str = "cosine",
                 device: Optional[str] = None, nlist: int = 64, nprobe: int = 16,
                 name: str = "default", persist_dir: Optional[str] = None,
                 batch_queries: Optional[bool] = None, hnsw_m: int = 16, hnsw_ef_construction: int = 200,
                 hnsw_ef: int = 64):
        self.embedder = embedder
        self.dim = dim
        self.name = name
        self.metric = metric
        self.index_type = index_type
        if index_type == "ivf_flat":
            self.index = IVFFlatIndex(dim, nlist, nprobe, metric, device)
        elif index_type == "hnsw":
            from .hnsw import HNSWIndex

            self.index = HNSWIndex(dim, metric, M=hnsw_m, ef_construction=hnsw_ef_construction, ef=hnsw_ef)
        else:
            self.index = FlatIndex(dim, metric, device)
        self.docs = DocStore()
        self.lock = threading.RLock()
        self._write_ev = None
        self._batcher = None
        dev = torch.device(device) if device is not None else self.index_device()
        # the query batcher groups searches on the GPU index's stream; a host-side HNSW graph
        # answers each query on the calling thread
        use = batch_queries if batch_queries is not None else (
            dev.type == "cuda" and self.index_device().type == "cuda"
            and os.environ.get("NGA_BATCH_QUERIES", "1") != "0")
        if use:
            # NGA_QUERY_BATCH_WAIT_MS: how long the first query of a batch waits for company
            self._batcher = _QueryBatcher(self, dev, wait_s=float(os.environ.get("NGA_QUERY_BATCH_WAIT_MS", "2")) / 1e3)
        self.persist_dir = persist_dir
        if persist_dir and (Path(persist_dir) / "index.json").exists():
            self.load(persist_dir)

    def __len__(self):
        return len(self.docs)

    # ------------------------------------------------------------------ write
    def add_texts(self, texts: Sequence[str], metadatas: Optional[Sequence[dict]] = None,
                  embeddings: Optional[torch.Tensor] = None) -> List[int]:
        texts = list(texts)
        if not texts:
            return []
        vecs = embeddings if embeddings is not None else _embed_docs(self.embedder, texts)
        with self.lock:
            ids = self.docs.new_ids(len(texts))
            self.index.add(vecs, torch.tensor(ids, dtype=torch.int64))
            self.docs.add(ids, texts, metadatas)
            self._mark_write()
        if self.persist_dir:
            self.save(self.persist_dir)
        return ids

    def add_documents(self, documents: Sequence[Document]) -> List[int]:
        return self.add_texts([d.page_content for d in documents], [d.metadata for d in documents])

    def delete(self, ids: Iterable[int]) -> int:
        ids = list(ids)
        with self.lock:
            n = self.index.remove(ids)
            self.docs.remove(ids)
            self._mark_write()
        if self.persist_dir:
            self.save(self.persist_dir)
        return n

    def delete_by_filename(self, filename: str) -> bool:
        ids = self.docs.ids_for("filename", filename) or self.docs.ids_for("source", filename)
        if not ids:
            return False
        self.delete(ids)
        return True

    def get_filenames(self) -> List[str]:
        out = self.docs.filenames()
        if not out:
            seen = []
            for m in self.docs.meta.values():
                s = m.get("source")
                if s and s not in seen:
                    seen.append(s)
            out = [os.path.basename(s) for s in seen]
        return out

    # ------------------------------------------------------------------ read
    def similarity_search_with_score_batch(self, queries: Sequence[str], k: int = 4
                                           ) -> List[List[Tuple[Document, float]]]:
        if len(self.docs) == 0:
            return [[] for _ in queries]
        q = _embed_queries(self.embedder, queries)
        with self.lock:
            vals, ids = self.index.search(q, k)
            vals, ids = vals.cpu().tolist(), ids.cpu().tolist()
            out = []
            for vs, ds in zip(vals, ids):
                row = []
                for v, d in zip(vs, ds):
                    if d < 0 or not self.docs.contains(d):
                        continue
                    row.append((Document(self.docs.get(d), dict(self.docs.metadata(d), doc_id=d)), float(v)))
                out.append(row)
        return out

    def similarity_search_with_score(self, query: str, k: int = 4) -> List[Tuple[Document, float]]:
        if self._batcher is not None:
            return self._batcher.submit(query, k).result()
        return self.similarity_search_with_score_batch([query], k)[0]

    def _mark_write(self):
        """Event after an index mutation: the query batcher's stream waits on it (and on
        nothing else, so searches never queue behind an LLM step on the default stream)."""
        if self._batcher is not None and torch.cuda.is_available() and self.index_device().type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
            self._write_ev = ev

    def index_device(self) -> torch.device:
        return torch.device(getattr(self.index, "device", "cpu"))

    def similarity_search(self, query: str, k: int = 4) -> List[Document]:
        return [d for d, _ in self.similarity_search_with_score(query, k)]

    def relevance(self, score: float) -> float:
        """Map a raw score to relevance like LangChain's euclidean relevance function for
        unit vectors, 1 - ||q - x|| / sqrt(2) (FAISS default store in the reference)."""
        if self.metric == "l2":
            return 1.0 - max(0.0, -score) ** 0.5 / 2 ** 0.5
        if self.metric == "cosine":
            return 1.0 - max(0.0, 2.0 - 2.0 * score) ** 0.5 / 2 ** 0.5
        return score

    def similarity_search_with_relevance_scores(self, query: str, k: int = 4,
                                                score_threshold: Optional[float] = None):
        res = [(d, self.relevance(s)) for d, s in self.similarity_search_with_score(query, k)]
        if score_threshold is not None:
            res = [(d, s) for d, s in res if s >= score_threshold]
        return res

    def as_retriever(self, search_type: str = "similarity", search_kwargs: Optional[dict] = None):
        return Retriever(self, search_type, search_kwargs or {})

    # ------------------------------------------------------------------ persistence
    def save(self, path: str):
        with self.lock:
            self.index.save(path)
            self.docs.save(path)
            (Path(path) / "store.json").write_text(json.dumps(
                {"name": self.name, "dim": self.dim, "metric": self.metric, "index_type": self.index_type}))

    def load(self, path: str):
        p = Path(path)
        kind = json.loads((p / "index.json").read_text()).get("kind", "flat")
        dev = str(self.index.device)
        if kind == "hnsw":
            from .hnsw import HNSWIndex

            self.index = HNSWIndex.load(path)
        else:
            self.index = IVFFlatIndex.load(path, dev) if kind == "ivf_flat" else FlatIndex.load(path, dev)
        self.docs = DocStore.load(path)


class Retriever:
    """``vs.as_retriever(search_type=..., search_kwargs={k, score_threshold})``."""

    def __init__(self, store: VectorStore, search_type: str, search_kwargs: dict):
        self.store = store
        self.search_type = search_type
        self.k = int(search_kwargs.get("k", 4))
        self.score_threshold = search_kwargs.get("score_threshold")

    def invoke(self, query: str) -> List[Document]:
        if self.search_type == "similarity_score_threshold":
            return [d for d, _ in self.store.similarity_search_with_relevance_scores(
                query, self.k, self.score_threshold)]
        return self.store.similarity_search(query, self.k)

    get_relevant_documents = invoke

    def invoke_with_scores(self, query: str):
        return self.store.similarity_search_with_score(query, self.k)


_STORES: Dict[str, VectorStore] = {}
_STORES_LOCK = threading.Lock()


def get_store(name: str, factory) -> VectorStore:
    with _STORES_LOCK:
        vs = _STORES.get(name)
        if vs is None:
            vs = factory(name)
            _STORES[name] = vs
        return vs


def reset_stores():
    with _STORES_LOCK:
        _STORES.clear()
