"""Vector-DB client facades with the reference's ``VectorClient`` contract, backed by the
in-HBM indices of this package instead of a Milvus or Qdrant server.

Reference: experimental/multimodal_assistant/retriever/vector.py:28-228 (also
RetrievalAugmentedGeneration/examples/multimodal_rag/retriever/vector.py:44, SURVEY.md
§2.A C10/E6). Its clients share one shape, kept here:

* ``create_collection(name, embedding_size)``;
* ``update(documents, embeddings, collection_name)``: Qdrant's ``upsert`` uses the
  document's position as point id (a re-upload replaces), Milvus' ``insert`` appends;
* ``search(query_vectors, limit) -> (concatdocs, sources)``, where ``concatdocs`` is
  ``"[[DOCUMENT i]]\\n\\n<content>\\n\\n"`` per hit (0-based for Milvus, 1-based for
  Qdrant, as in the reference) and ``sources`` maps ``metadata["source"]`` to
  ``{"doc_content", "doc_metadata"}``.

``MilvusStyleClient`` uses IVF-Flat with the reference defaults (L2, nlist 100, nprobe 5).
``QdrantStyleClient`` uses a flat cosine index. Collections live in a process-wide
registry, the analogue of the server, so several clients see the same collection.
"""
from __future__ import annotations

import threading
from abc import ABC, abstractmethod
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch

from .flat import FlatIndex
from .ivf import IVFFlatIndex


@dataclass
class _Collection:
    index: Any
    dim: int
    payloads: Dict[int, dict] = field(default_factory=dict)


_REGISTRY: Dict[str, _Collection] = {}
_LOCK = threading.Lock()


def drop_collection(name: str) -> None:
    with _LOCK:
        _REGISTRY.pop(name, None)


def has_collection(name: str) -> bool:
    return name in _REGISTRY


class VectorClient(ABC):
    def __init__(self, collection_name: str = "collection", embedding_size: int = 1024,
                 device: Optional[str] = None):
        self.collection_name = collection_name
        self.embedding_size = embedding_size
        self.device = device
        if not has_collection(collection_name):
            self.create_collection(collection_name, embedding_size)

    @abstractmethod
    def _new_index(self, dim: int):
        ...

    def create_collection(self, collection_name: str, embedding_size: int) -> None:
        with _LOCK:
            if collection_name not in _REGISTRY:
                _REGISTRY[collection_name] = _Collection(self._new_index(embedding_size), embedding_size)

    def _col(self, name: Optional[str] = None) -> _Collection:
        return _REGISTRY[name or self.collection_name]

    def update(self, documents: Sequence, embeddings, collection_name: Optional[str] = None) -> None:
        name = collection_name or self.collection_name
        if not has_collection(name):
            self.create_collection(name, self.embedding_size)
        col = self._col(name)
        vecs = torch.as_tensor(embeddings, dtype=torch.float32)
        with _LOCK:
            ids = self._ids_for(col, len(documents))
            col.index.add(vecs, ids)
            for i, d in zip(ids.tolist(), documents):
                col.payloads[i] = {"content": d.page_content, "metadata": dict(d.metadata)}

    def _ids_for(self, col: _Collection, n: int) -> torch.Tensor:
        """Milvus ``insert``: append (fresh primary keys)."""
        start = max(col.payloads) + 1 if col.payloads else 0
        return torch.arange(start, start + n, dtype=torch.int64)

    def _hits(self, query_vectors, limit: int) -> List[Tuple[int, float]]:
        q = torch.as_tensor(query_vectors, dtype=torch.float32)
        if q.dim() == 1:
            q = q.unsqueeze(0)
        col = self._col()
        if len(col.index) == 0:
            return []
        scores, ids = col.index.search(q[:1], limit)
        return [(int(i), float(s)) for s, i in zip(scores[0].tolist(), ids[0].tolist()) if i >= 0]

    def search(self, query_vectors, limit: int = 5) -> Tuple[str, Dict[str, dict]]:
        concatdocs, sources = "", {}
        col = self._col()
        for rank, (i, _) in enumerate(self._hits(query_vectors, limit)):
            p = col.payloads.get(i)
            if p is None:
                continue
            meta = p["metadata"]
            sources[meta.get("source", str(i))] = {"doc_content": p["content"], "doc_metadata": meta}
            concatdocs += f"[[DOCUMENT {rank + self._first_label}]]\n\n" + p["content"] + "\n\n"
        return concatdocs, sources

    _first_label = 0

    def disconnect(self) -> None:
        pass


class MilvusStyleClient(VectorClient):
    """Milvus ``Collection`` with an IVF_FLAT index (metric L2, nlist 100, nprobe 5)."""

    metric_type = "L2"
    index_type = "IVF_FLAT"
    nlist = 100
    nprobe = 5
    _first_label = 0

    def _new_index(self, dim: int):
        return IVFFlatIndex(dim, nlist=self.nlist, nprobe=self.nprobe, metric="l2", device=self.device)


class QdrantStyleClient(VectorClient):
    """Qdrant collection with ``Distance.COSINE``; ``update`` upserts by point id."""

    _first_label = 1

    def _new_index(self, dim: int):
        return FlatIndex(dim, "cosine", self.device)

    def _ids_for(self, col: _Collection, n: int) -> torch.Tensor:
        """Qdrant ``upsert`` with ``PointStruct(id=i)``: point i is replaced."""
        ids = torch.arange(n, dtype=torch.int64)
        if len(col.index):
            col.index.remove(ids.tolist())
        return ids
