"""Canonical QA chatbot (RetrievalAugmentedGeneration/examples/developer_rag/chains.py).

ingest: load (PDF text layer / text) -> token splitter (chunk_size-2, overlap 200) -> embed
passages -> in-HBM index, metadata ``{"filename": <name minus 4 chars>, "common_field": "all"}``.
rag: retrieve top_k -> drop nodes past 1500 tokens (LimitRetrievedNodesLength) -> the
``rag_template`` filled with context/query as one user message -> streamed answer.

Kept quirks: the stored filename drops the last 4 characters (``filename[:-4]``, reference
chains.py:86), and ``document_search`` labels every chunk with the first chunk's filename
(chains.py:191). Fixed on purpose: the reference retrieves twice per question (once as a
check, once inside the query engine, chains.py:156,172); here the first retrieval is reused.
"""
from __future__ import annotations

import logging
from typing import Any, Dict, Generator, List

from ...chain_server import utils
from ...chain_server.base import BaseExample
from ..common import NO_CONTEXT, TracedExample, ingest_file

logger = logging.getLogger(__name__)


class QAChatbot(BaseExample, TracedExample):
    def __init__(self):
        TracedExample.__init__(self)

    def ingest_docs(self, filepath: str, filename: str):
        try:
            logger.info("Ingesting %s in vectorDB", filename)
            vs = utils.get_vectorstore()
            ingest_file(vs, filepath, filename, metadata={"filename": filename[:-4], "common_field": "all"})
            logger.info("Document %s ingested successfully", filename)
        except Exception as e:
            logger.error("Failed to ingest document due to exception %s", e)
            raise ValueError("Failed to upload document. Please upload an unstructured text document.")

    def get_documents(self) -> List[str]:
        return utils.get_docs_vectorstore(utils.get_vectorstore())

    def delete_documents(self, filenames: List[str]) -> bool:
        return utils.del_docs_vectorstore(utils.get_vectorstore(), filenames)

    def llm_chain(self, query: str, chat_history: List[Any], **kwargs) -> Generator[str, None, None]:
        logger.info("Using llm to generate response directly without knowledge base.")
        prompt = utils.get_config().prompts.chat_template
        messages = [("system", prompt), ("user", query)]
        return self.stream_llm(messages, **kwargs)

    def rag_chain(self, query: str, chat_history: List[Any], **kwargs) -> Generator[str, None, None]:
        logger.info("Using rag to generate response from document")
        cfg = utils.get_config()
        vs = utils.get_vectorstore()
        hits = self.retrieve(vs, query, cfg.retriever.top_k)
        if not hits:
            logger.warning("Retrieval failed to get any relevant context")
            return iter([NO_CONTEXT])
        docs = utils.LimitRetrievedNodesLength().postprocess([d for d, _ in hits])
        context = "\n\n".join(d.page_content for d in docs)
        prompt = cfg.prompts.rag_template.replace("{context_str}", context).replace("{query_str}", query)
        return self.stream_llm([("user", prompt)], **kwargs)

    def document_search(self, content: str, num_docs: int) -> List[Dict[str, Any]]:
        try:
            hits = self.retrieve(utils.get_vectorstore(), content, utils.get_config().retriever.top_k)
            if not hits:
                return []
            first = hits[0][0].metadata.get("filename", "")
            return [{"score": s, "source": first, "content": d.page_content} for d, s in hits]
        except Exception as e:  # noqa: BLE001
            logger.error("Error from /documentSearch endpoint. Error details: %s", e)
            return []
