"""Host-side document store for the vector index: id -> (text, metadata), plus a cache of
each chunk's LLM token ids so prompts are assembled without re-tokenising context.

Covers the reference's per-backend document bookkeeping (``get_docs_vectorstore_*`` /
``del_docs_vectorstore_*``, RetrievalAugmentedGeneration/common/utils.py:334-468): list the
source filenames, delete every chunk of a filename. Persistence is a JSONL file written
atomically next to the index snapshot.
"""
from __future__ import annotations

import json
import os
import threading
from pathlib import Path
from typing import Dict, Iterable, List, Optional

from ..utils.synthetic import TextGen


class DocStore:
    def __init__(self):
        self.texts: Dict[int, str] = {}
        self.meta: Dict[int, dict] = {}
        self._tok_cache: Dict[int, List[int]] = {}
        self._sep: Optional[List[int]] = None
        self.lock = threading.RLock()
        self._next = 0

    def __len__(self):
        return len(self.texts)

    def new_ids(self, n: int) -> List[int]:
        with self.lock:
            s = self._next
            self._next += n
            return list(range(s, s + n))

    def add(self, ids: Iterable[int], texts: Iterable[str], metas: Optional[Iterable[dict]] = None):
        with self.lock:
            metas = list(metas) if metas is not None else None
            for j, (i, t) in enumerate(zip(ids, texts)):
                self.texts[int(i)] = t
                self.meta[int(i)] = dict(metas[j]) if metas else {}
                self._tok_cache.pop(int(i), None)
                self._next = max(self._next, int(i) + 1)

    def get(self, i: int) -> str:
        return self.texts[int(i)]

    def contains(self, i: int) -> bool:
        return int(i) in self.texts

    def metadata(self, i: int) -> dict:
        return self.meta.get(int(i), {})

    def token_ids(self, i: int, tok) -> List[int]:
        c = self._tok_cache.get(i)
        if c is None:
            c = tok.encode(self.get(i))
            self._tok_cache[i] = c
        return c

    def sep_ids(self, tok) -> List[int]:
        if self._sep is None:
            self._sep = tok.encode("\n\n")
        return self._sep

    def ids_for(self, key: str, value: str) -> List[int]:
        with self.lock:
            return [i for i, m in self.meta.items() if m.get(key) == value]

    def filenames(self) -> List[str]:
        with self.lock:
            seen, out = set(), []
            for m in self.meta.values():
                f = m.get("filename")
                if f and f not in seen:
                    seen.add(f)
                    out.append(f)
            return out

    def remove(self, ids: Iterable[int]):
        with self.lock:
            for i in ids:
                self.texts.pop(int(i), None)
                self.meta.pop(int(i), None)
                self._tok_cache.pop(int(i), None)

    def save(self, path: str):
        p = Path(path)
        p.mkdir(parents=True, exist_ok=True)
        tmp = p / "docstore.jsonl.tmp"
        with self.lock, open(tmp, "w") as f:
            for i, t in self.texts.items():
                f.write(json.dumps({"id": i, "text": t, "meta": self.meta.get(i, {})}) + "\n")
        os.replace(tmp, p / "docstore.jsonl")

    @classmethod
    def load(cls, path: str) -> "DocStore":
        ds = cls()
        f = Path(path) / "docstore.jsonl"
        if f.exists():
            with open(f) as fh:
                for line in fh:
                    r = json.loads(line)
                    ds.add([r["id"]], [r["text"]], [r.get("meta", {})])
        return ds


class SyntheticDocStore(DocStore):
    """A docstore over n synthetic chunks backed by a fixed pool of generated texts
    (doc i = pool[i % pool_size] tagged with its id), for 1M-10M-chunk benchmark indices."""

    def __init__(self, n_docs: int, pool_size: int = 2048, words_per_chunk: int = 470, seed: int = 0):
        super().__init__()
        g = TextGen(seed)
        self.pool = []
        for _ in range(pool_size):
            ws = []
            while len(ws) < words_per_chunk:
                ws += g.sentence().split()
            self.pool.append(" ".join(ws[:words_per_chunk]))
        self.n_docs = n_docs
        self._pool_tok: Dict[int, List[int]] = {}
        self._next = n_docs

    def __len__(self):
        return self.n_docs + len(self.texts)

    def contains(self, i: int) -> bool:
        i = int(i)
        return 0 <= i < self.n_docs or i in self.texts

    def get(self, i: int) -> str:
        i = int(i)
        if i in self.texts:
            return self.texts[i]
        return f"[doc {i}] " + self.pool[i % len(self.pool)]

    def metadata(self, i: int) -> dict:
        i = int(i)
        return self.meta.get(i, {"filename": f"synthetic_{i // 1000}.txt"})

    def token_ids(self, i: int, tok) -> List[int]:
        i = int(i)
        if i in self.texts:
            return super().token_ids(i, tok)
        k = i % len(self.pool)
        c = self._pool_tok.get(k)
        if c is None:
            c = tok.encode(self.pool[k])
            self._pool_tok[k] = c
        return c
