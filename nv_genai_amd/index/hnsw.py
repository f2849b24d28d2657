"""HNSW proximity-graph index (Milvus ``index_type: HNSW`` with ``M`` / ``efConstruction``, the
index of the reference's streaming-ingest collections:
experimental/streaming_ingest_rag/morpheus_examples/streaming_ingest_rag/vdb_upload/kafka_config.yaml:112-122).

The graph lives in host memory and is built and searched by the native runtime
(``csrc/runtime/hnsw.cpp``; adds link a batch with worker threads, searches release the GIL
and split a query batch over threads).
Same interface and score convention as :class:`~nv_genai_amd.index.flat.FlatIndex` —
``search`` returns (scores, ids) with scores = -squared L2, or the inner product (cosine: of
the normalised vectors), and -1 ids for missing results — so ``VectorStore(index_type="hnsw")``
swaps it in. On MI355X the flat / IVF scan in HBM is the throughput path for query batches;
HNSW answers single queries on the host with no kernel launch and no device round trip.
"""
from __future__ import annotations

import json
import os
from pathlib import Path
from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from .. import _rt


class HNSWIndex:
    def __init__(self, dim: int, metric: str = "cosine", M: int = 16, ef_construction: int = 200,
                 ef: int = 64, threads: Optional[int] = None, seed: int = 100, _graph=None):
        if metric not in ("cosine", "ip", "l2"):
            raise ValueError("metric must be cosine, ip or l2")
        self.dim, self.metric = int(dim), metric
        self.M, self.ef_construction = int(M), int(ef_construction)
        self.threads = threads or min(16, os.cpu_count() or 1)
        self.g = _graph if _graph is not None else _rt.HNSW(self.dim, metric, self.M, self.ef_construction,
                                                            int(ef), int(seed))
        self.device = torch.device("cpu")

    def __len__(self) -> int:
        return len(self.g)

    @property
    def ef(self) -> int:
        return self.g.ef

    @ef.setter
    def ef(self, v: int) -> None:
        self.g.ef = int(v)

    @staticmethod
    def _np(x) -> np.ndarray:
        if isinstance(x, torch.Tensor):
            x = x.detach().to("cpu", torch.float32).numpy()
        return np.ascontiguousarray(np.asarray(x, dtype=np.float32))

    def add(self, vecs, ids) -> None:
        v = self._np(vecs)
        if v.ndim == 1:
            v = v[None]
        i = np.ascontiguousarray(np.asarray(ids.cpu() if isinstance(ids, torch.Tensor) else ids, dtype=np.int64))
        self.g.add(v, i, self.threads)

    def remove(self, ids: Sequence[int]) -> int:
        return int(self.g.remove([int(i) for i in ids]))

    def search(self, q, k: int, ef: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        qa = self._np(q)
        if qa.ndim == 1:
            qa = qa[None]
        s, i = self.g.search(qa, int(k), int(ef or 0), self.threads)
        return torch.from_numpy(s), torch.from_numpy(i)

    # ------------------------------------------------------------------ persistence
    def save(self, path: str) -> None:
        p = Path(path)
        p.mkdir(parents=True, exist_ok=True)
        tmp = p / "graph.hnsw.tmp"
        self.g.save(str(tmp))
        os.replace(tmp, p / "graph.hnsw")
        (p / "index.json").write_text(json.dumps({"dim": self.dim, "metric": self.metric, "kind": "hnsw",
                                                  "M": self.M, "ef_construction": self.ef_construction,
                                                  "n": len(self)}))

    @classmethod
    def load(cls, path: str, device: Optional[str] = None) -> "HNSWIndex":
        p = Path(path)
        meta = json.loads((p / "index.json").read_text())
        g = _rt.HNSW.load(str(p / "graph.hnsw"))
        return cls(meta["dim"], meta["metric"], meta["M"], meta["ef_construction"], g.ef, _graph=g)
