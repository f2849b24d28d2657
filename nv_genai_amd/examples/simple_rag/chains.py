"""Minimal example from the "simple example" tutorial (SURVEY.md §2.A C17;
docs/simple-example/code/api-catalog/{boilerplate,ingest,llm,rag,documents}/chains.py):
the smallest complete BaseExample — text/PDF ingest, plain LLM chat, RAG with the
"Context / Question" prompt, search, list and delete.
"""
from __future__ import annotations

import logging
import os
from typing import Any, Dict, Generator, List

from ...chain_server import utils
from ...chain_server.base import BaseExample
from ..common import TracedExample, ingest_file

logger = logging.getLogger(__name__)


class SimpleExample(BaseExample, TracedExample):
    def __init__(self):
        TracedExample.__init__(self)

    def ingest_docs(self, filepath: str, filename: str) -> None:
        ingest_file(utils.get_vectorstore(), filepath, filename)

    def llm_chain(self, query: str, chat_history: List[Any], **kwargs) -> Generator[str, None, None]:
        return self.stream_llm([("system", "You are a helpful AI assistant."), ("user", query)], **kwargs)

    def rag_chain(self, query: str, chat_history: List[Any], **kwargs) -> Generator[str, None, None]:
        hits = self.retrieve(utils.get_vectorstore(), query, 4)
        context = "\n\n".join(d.page_content for d, _ in hits)
        prompt = f"Answer solely based on the following context:\n<Documents>\n{context}\n</Documents>\n\nQuestion: {query}"
        return self.stream_llm([("system", "You are a helpful AI assistant."), ("user", prompt)], **kwargs)

    def document_search(self, content: str, num_docs: int) -> List[Dict[str, Any]]:
        hits = self.retrieve(utils.get_vectorstore(), content, num_docs)
        return [{"source": os.path.basename(d.metadata.get("source", "")), "content": d.page_content, "score": s}
                for d, s in hits]

    def get_documents(self) -> List[str]:
        return utils.get_docs_vectorstore(utils.get_vectorstore())

    def delete_documents(self, filenames: List[str]) -> bool:
        return utils.del_docs_vectorstore(utils.get_vectorstore(), filenames)
