"""Deterministic stand-ins for contract tests and GPU-less plumbing (SURVEY.md §4 "fake /
substitute backends": the reference's own ``random_embedding`` fake embedder,
knowledge_graph_rag/vectorstore/search.py:44-49, and the LocalLLM("gpt2") self-test).

* :class:`HashEmbeddings` — feature-hashed bag of words, L2-normalised: texts sharing words
  have high cosine similarity, so retrieval behaves sensibly with no model at all.
* :class:`FakeChatModel` — streams a deterministic, prompt-dependent answer word by word;
  can be told to fail (fault injection for error-frame tests).
"""
from __future__ import annotations

import hashlib
import re
from typing import Iterator, List, Optional, Sequence

import torch

from .local import Messages, normalize_messages

_WORD = re.compile(r"[A-Za-z0-9]+")


class HashEmbeddings:
    def __init__(self, dim: int = 256, model: str = "hash-embed"):
        self.dim = dim
        self.model = model

    def _vec(self, text: str) -> torch.Tensor:
        v = torch.zeros(self.dim)
        for w in _WORD.findall(text.lower()):
            h = int.from_bytes(hashlib.blake2b(w.encode(), digest_size=8).digest(), "little")
            v[h % self.dim] += 1.0 if (h >> 63) == 0 else -1.0
        n = v.norm()
        if n == 0:
            v[0] = 1.0
            n = 1.0
        return v / n

    def embed(self, texts: Sequence[str], input_type: str = "passage", truncate: str = "END") -> torch.Tensor:
        return torch.stack([self._vec(t) for t in texts]) if texts else torch.zeros(0, self.dim)

    def embed_query(self, text: str) -> List[float]:
        return self._vec(text).tolist()

    def embed_documents(self, texts: Sequence[str]) -> List[List[float]]:
        return self.embed(texts).tolist()

    def embed_query_tensor(self, texts):
        return self.embed(texts, "query")

    def embed_documents_tensor(self, texts):
        return self.embed(texts, "passage")


class FakeChatModel:
    def __init__(self, model: str = "fake-llm", fail: bool = False, words: int = 12, **defaults):
        self.model = model
        self.fail = fail
        self.words = words
        self.defaults = defaults
        self.calls: List[List[dict]] = []

    def stream(self, messages: Messages, **kw) -> Iterator[str]:
        msgs = normalize_messages(messages)
        self.calls.append(msgs)
        if self.fail:
            raise RuntimeError("injected LLM failure")
        last = msgs[-1]["content"] if msgs else ""
        h = hashlib.sha256(last.encode()).hexdigest()
        n = int(kw.get("max_tokens") or self.words)
        n = min(n, self.words)
        for i in range(n):
            yield (" " if i else "") + f"w{h[i % 64]}{i}"

    def invoke(self, messages: Messages, **kw) -> str:
        return "".join(self.stream(messages, **kw))

    __call__ = invoke

    def bind(self, **kw):
        return self
