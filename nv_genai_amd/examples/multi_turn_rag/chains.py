"""Multi-turn RAG with conversation memory (SURVEY.md §2.A C8;
RetrievalAugmentedGeneration/examples/multi_turn_rag/chains.py).

Two collections: documents (``COLLECTION_NAME``) and ``conv_store``. For each question both
are searched (score-threshold retrieval), the ``multi_turn_rag_template`` is filled with
{input} / {history} / {context} (+ "User Query: ..."), the answer streams, and the Q/A pair is
written back to ``conv_store`` ("User previously responded with ...", "Agent previously
responded with ...").

Kept quirk: ``rag_chain`` is a generator (it yields), so the reference's early
``return iter([...])`` paths yield nothing at all — an empty-retrieval question produces an
empty answer stream.
"""
from __future__ import annotations

import logging
from typing import Any, Generator, List

from ...chain_server import utils
from ...chain_server.base import BaseExample
from ..common import NO_CONTEXT, TracedExample, context_from, ingest_file

logger = logging.getLogger(__name__)


class MultiTurnChatbot(BaseExample, TracedExample):
    def __init__(self):
        TracedExample.__init__(self)

    def save_memory_and_get_output(self, d, vstore):
        vstore.add_texts([f"User previously responded with {d.get('input')}",
                          f"Agent previously responded with {d.get('output')}"])
        return d.get("output")

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
        return self.stream_llm([("system", cfg.prompts.chat_template), ("user", query)], **kwargs)

    def rag_chain(self, query: str, chat_history: List[Any], **kwargs) -> Generator[str, None, None]:
        cfg = utils.get_config()
        convstore = utils.get_vectorstore("conv_store")
        try:
            ds = utils.get_vectorstore()
            k, thr = cfg.retriever.top_k, cfg.retriever.score_threshold
            ctx_docs = [d for d, _ in self.retrieve(ds, query, k, thr)]
            hist_docs = [d for d, _ in self.retrieve(convstore, query, k, thr)]
            if not ctx_docs and not hist_docs:
                logger.warning("Retrieval failed to get any relevant context")
                return iter([NO_CONTEXT])  # yields nothing: this function is a generator
            prompt = (cfg.prompts.multi_turn_rag_template
                      .replace("{input}", query)
                      .replace("{history}", context_from(hist_docs))
                      .replace("{context}", context_from(ctx_docs))) + "User Query: " + query
            resp = ""
            for chunk in self.stream_llm([("user", prompt)], **kwargs):
                resp += chunk
                yield chunk
            self.save_memory_and_get_output({"input": query, "output": resp}, convstore)
        except Exception as e:  # noqa: BLE001
            logger.warning("Failed to generate response due to exception %s", e)
            return

    def document_search(self, content: str, num_docs: int):
        cfg = utils.get_config()
        hits = self.retrieve(utils.get_vectorstore(), content, cfg.retriever.top_k, cfg.retriever.score_threshold)
        import os

        return [{"source": os.path.basename(d.metadata.get("source", "")), "content": d.page_content, "score": s}
                for d, s in hits]

    def get_documents(self) -> List[str]:
        return utils.get_docs_vectorstore(utils.get_vectorstore())

    def delete_documents(self, filenames: List[str]) -> bool:
        return utils.del_docs_vectorstore(utils.get_vectorstore(), filenames)
