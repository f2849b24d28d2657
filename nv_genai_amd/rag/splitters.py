"""Text splitters, windowing done in the native runtime (``_rt``).

* :class:`TokenTextSplitter` — SentenceTransformersTokenTextSplitter semantics: windows of
  ``tokens_per_chunk`` encoder tokens (the reference passes ``chunk_size - 2`` to leave room
  for [CLS]/[SEP], RetrievalAugmentedGeneration/common/utils.py:321-331) overlapping by
  ``chunk_overlap`` tokens, decoded back to text.
* :class:`RecursiveCharacterTextSplitter` / :class:`CharacterTextSplitter` — character
  windows over a separator hierarchy (multimodal_rag 1000/100, query_decomposition_rag).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

from .._native import rt
from ..index.vectorstore import Document


class TokenTextSplitter:
    def __init__(self, tokens_per_chunk: int = 508, chunk_overlap: int = 200, tokenizer=None):
        from ..utils.tokenizer import embed_tokenizer

        self.tokens_per_chunk = tokens_per_chunk
        self.chunk_overlap = chunk_overlap
        self.tok = tokenizer or embed_tokenizer()

    def split_text(self, text: str) -> List[str]:
        enc = self.tok.tok.encode(text, add_special_tokens=False)
        ids, offs = enc.ids, enc.offsets
        if not ids:
            return []
        out = []
        for s, e in rt.token_windows(len(ids), self.tokens_per_chunk, self.chunk_overlap):
            a, b = offs[s][0], offs[e - 1][1]
            chunk = text[a:b].strip()
            if chunk:
                out.append(chunk)
        return out

    def split_documents(self, docs: Sequence[Document]) -> List[Document]:
        return [Document(c, dict(d.metadata)) for d in docs for c in self.split_text(d.page_content)]

    def count_tokens(self, text: str) -> int:
        return len(self.tok.tok.encode(text, add_special_tokens=False).ids)


class RecursiveCharacterTextSplitter:
    def __init__(self, chunk_size: int = 1000, chunk_overlap: int = 100,
                 separators: Optional[List[str]] = None):
        self.chunk_size = chunk_size
        self.chunk_overlap = chunk_overlap
        self.separators = separators or ["\n\n", "\n", " ", ""]

    def split_text(self, text: str) -> List[str]:
        return rt.char_split(text, self.chunk_size, self.chunk_overlap, self.separators)

    def split_documents(self, docs: Sequence[Document]) -> List[Document]:
        return [Document(c, dict(d.metadata)) for d in docs for c in self.split_text(d.page_content)]


class CharacterTextSplitter(RecursiveCharacterTextSplitter):
    def __init__(self, chunk_size: int = 1000, chunk_overlap: int = 0, separator: str = "\n\n"):
        super().__init__(chunk_size, chunk_overlap, [separator, ""])
