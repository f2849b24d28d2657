"""LangChain-style text QA chatbot (SURVEY.md §2.A C7;
RetrievalAugmentedGeneration/examples/nvidia_api_catalog/chains.py).

ingest: only .txt/.pdf/.md; load -> token splitter -> add_documents.
rag: ``similarity_score_threshold`` retrieval (k = top_k, threshold = score_threshold; the
reference falls back to plain similarity when the store cannot threshold — this store can),
context = chunks joined with blank lines, ``rag_template`` as the system message and
"Context: ...\\n\\nQuestion: ...\\n" as the user message. Chat history is ignored (the
reference resets it to []).
"""
from __future__ import annotations

import logging
import os
from typing import Any, Dict, Generator, List

from ...chain_server import utils
from ...chain_server.base import BaseExample
from ..common import NO_CONTEXT, NO_DOCS, TracedExample, context_from, ingest_file

logger = logging.getLogger(__name__)


class NvidiaAPICatalog(BaseExample, TracedExample):
    def __init__(self):
        TracedExample.__init__(self)

    def ingest_docs(self, filepath: str, filename: str):
        if not filename.endswith((".txt", ".pdf", ".md")):
            raise ValueError(f"{filename} is not a valid Text, PDF or Markdown file")
        try:
            ingest_file(utils.get_vectorstore(), filepath, filename)
        except Exception as e:
            logger.error("Failed to ingest document due to exception %s", e)
            raise ValueError("Failed to upload document. Please upload an unstructured text document.")

    def llm_chain(self, query: str, chat_history: List[Any], **kwargs) -> Generator[str, None, None]:
        cfg = utils.get_config()
        messages = [("system", cfg.prompts.chat_template), ("user", "\n\nQuestion: " + query + "\n")]
        return self.stream_llm(messages, **kwargs)

    def _docs(self, query: str):
        cfg = utils.get_config()
        hits = self.retrieve(utils.get_vectorstore(), query, cfg.retriever.top_k, cfg.retriever.score_threshold)
        return [d for d, _ in hits]

    def rag_chain(self, query: str, chat_history: List[Any], **kwargs) -> Generator[str, None, None]:
        cfg = utils.get_config()
        try:
            docs = self._docs(query)
            if not docs:
                logger.warning("Retrieval failed to get any relevant context")
                return iter([NO_CONTEXT])
            user = "Context: " + context_from(docs) + "\n\nQuestion: " + query + "\n"
            return self.stream_llm([("system", cfg.prompts.rag_template), ("user", user)], **kwargs)
        except Exception as e:  # noqa: BLE001
            logger.warning("Failed to generate response due to exception %s", e)
        return iter([NO_DOCS])

    def document_search(self, content: str, num_docs: int) -> List[Dict[str, Any]]:
        try:
            cfg = utils.get_config()
            hits = self.retrieve(utils.get_vectorstore(), content, cfg.retriever.top_k, cfg.retriever.score_threshold)
            return [{"source": os.path.basename(d.metadata.get("source", "")), "content": d.page_content, "score": s}
                    for d, s in hits]
        except Exception as e:  # noqa: BLE001
            logger.error("Error from POST /search endpoint. Error details: %s", e)
            return []

    def get_documents(self) -> List[str]:
        return utils.get_docs_vectorstore(utils.get_vectorstore())

    def delete_documents(self, filenames: List[str]) -> bool:
        return utils.del_docs_vectorstore(utils.get_vectorstore(), filenames)
