"""The example plugin contract (RetrievalAugmentedGeneration/common/base.py:21-33,
docs/simple-examples.md:44-62).

The chain server discovers the first class in the example directory that has
``ingest_docs``, ``llm_chain`` and ``rag_chain`` and instantiates it per request. The server
calls ``llm_chain(query, chat_history, **llm_settings)`` / ``rag_chain(...)`` — both return a
generator of text chunks — and the optional ``document_search``, ``get_documents`` and
``delete_documents`` hooks.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Any, Dict, Generator, List


class BaseExample(ABC):
    @abstractmethod
    def llm_chain(self, query: str, chat_history: List[Any], **kwargs) -> Generator[str, None, None]:
        """Answer without retrieval."""

    @abstractmethod
    def rag_chain(self, query: str, chat_history: List[Any], **kwargs) -> Generator[str, None, None]:
        """Answer with retrieval from the knowledge base."""

    @abstractmethod
    def ingest_docs(self, filepath: str, filename: str) -> None:
        """Split, embed and index one uploaded file."""

    def document_search(self, content: str, num_docs: int) -> List[Dict[str, Any]]:
        """Return [{"content", "source", "score"}] for the query."""
        raise NotImplementedError

    def get_documents(self) -> List[str]:
        raise NotImplementedError

    def delete_documents(self, filenames: List[str]) -> bool:
        raise NotImplementedError
