"""Helpers shared by the example chains: traced LLM streaming, ingestion, retrieval."""
from __future__ import annotations

import logging
import uuid
from typing import Iterator, List, Optional, Sequence

from ..chain_server import utils
from ..observability.tracing import TracingCallback, get_tracer
from ..rag.loaders import load_file

log = logging.getLogger(__name__)
NO_CONTEXT = "No response generated from LLM, make sure your query is relavent to the ingested document."
NO_DOCS = "No response generated from LLM, make sure you have ingested document from the Knowledge Base Tab."


class LLMStream:
    """A traced LLM answer stream. Iterating it synchronously is the reference behaviour (a
    generator of text chunks). With an in-process engine it also iterates asynchronously:
    the chain server then forwards tokens from the engine's asyncio queue with no thread per
    stream, coalescing the tokens that arrived since the last frame."""

    def __init__(self, cb, llm, messages, kwargs):
        self.cb, self.llm, self.messages, self.kwargs = cb, llm, messages, kwargs
        self.rid = uuid.uuid4().hex
        self._handle = None

    def prepare(self) -> "LLMStream":
        """Tokenise the prompt and queue it on the engine now (the chain server calls this on
        the request's worker thread, so chat-template encoding stays off the event loop and
        the request enters the scheduler as soon as its context is ready)."""
        if self._handle is None and self.supports_async and hasattr(self.llm, "submit"):
            self._handle = self.llm.submit(self.messages)
        return self

    def cancel(self) -> None:
        """Abort the request ``prepare`` queued if its stream never finished being consumed
        (the chain server runs this after every response: a client that disconnects before
        the body starts would otherwise leave the request decoding to max_tokens)."""
        h = self._handle
        if h is not None and not h.done.is_set():
            h.cancel()

    def _start(self):
        self.cb.on_llm_start(self.rid, self.messages, **{k: v for k, v in self.kwargs.items() if v is not None})

    def __iter__(self) -> Iterator[str]:
        self._start()
        out: List[str] = []
        try:
            for chunk in self.llm.stream(self.messages):
                self.cb.on_llm_new_token(self.rid, chunk)
                out.append(chunk)
                yield chunk
        except Exception as e:
            self.cb.on_llm_error(self.rid, e)
            raise
        self.cb.on_llm_end(self.rid, "".join(out))

    @property
    def supports_async(self) -> bool:
        return hasattr(self.llm, "astream")

    async def __aiter__(self):
        self._start()
        out: List[str] = []
        try:
            async for chunk in self.llm.astream(self.messages, coalesce=True, handle=self._handle):
                self.cb.on_llm_new_token(self.rid, chunk)
                out.append(chunk)
                yield chunk
        except Exception as e:
            self.cb.on_llm_error(self.rid, e)
            raise
        self.cb.on_llm_end(self.rid, "".join(out))


class TracedExample:
    """Gives every example a callback handler (the reference's
    ``langchain_instrumentation_class_wrapper`` sets ``self.cb_handler``)."""

    def __init__(self):
        self.cb_handler = TracingCallback(get_tracer("chain-server"))

    def stream_llm(self, messages, **kwargs) -> "LLMStream":
        return LLMStream(self.cb_handler, utils.get_llm(**kwargs), messages, kwargs)

    def invoke_llm(self, messages, **kwargs) -> str:
        return "".join(self.stream_llm(messages, **kwargs))

    def retrieve(self, vs, query: str, k: int, threshold: Optional[float] = None):
        rid = uuid.uuid4().hex
        self.cb_handler.on_retriever_start(rid, query)
        if threshold is None:
            res = vs.similarity_search_with_score(query, k)
        else:
            res = vs.similarity_search_with_relevance_scores(query, k, threshold)
        self.cb_handler.on_retriever_end(rid, res)
        return res


def ingest_file(vs, filepath: str, filename: str, splitter=None, metadata: Optional[dict] = None,
                allowed: Optional[Sequence[str]] = None) -> int:
    if allowed is not None and not filename.lower().endswith(tuple(allowed)):
        raise ValueError(f"{filename} is not a valid Text, PDF or Markdown file")
    docs = load_file(filepath, filename)
    if not docs:
        log.warning("No documents available to process!")
        return 0
    for d in docs:
        d.metadata.update(metadata or {})
    splitter = splitter or utils.get_text_splitter()
    chunks = splitter.split_documents(docs)
    vs.add_documents(chunks)
    return len(chunks)


def context_from(docs, sep: str = "\n\n") -> str:
    return "".join(d.page_content + sep for d in docs)
