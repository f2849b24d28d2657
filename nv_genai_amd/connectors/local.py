"""In-process connector objects with the LangChain-style surface the reference's chains use
(``ChatNVIDIA.stream/invoke``, ``NVIDIAEmbeddings.embed_query/embed_documents``,
``NVIDIARerank``) — backed directly by the engines on this GPU, no HTTP hop.

``langchain`` / ``llama_index`` are not installed in this environment; these classes are the
framework's own minimal equivalents. The HTTP twins in
:mod:`nv_genai_amd.connectors.http` talk to the model server with the same methods.
"""
from __future__ import annotations

from typing import Iterator, List, Optional, Sequence, Union

from ..engine.llm_engine import SamplingParams
from ..serving.engine_service import EngineService, StreamHandle

Messages = Union[str, Sequence[dict], Sequence[tuple]]


def normalize_messages(messages: Messages) -> List[dict]:
    """Accept a plain prompt, [{"role", "content"}], or LangChain-style (role, content) tuples."""
    if isinstance(messages, str):
        return [{"role": "user", "content": messages}]
    out = []
    for m in messages:
        if isinstance(m, dict):
            out.append({"role": m.get("role", "user"), "content": m.get("content", "")})
        elif isinstance(m, (tuple, list)) and len(m) == 2:
            role = {"human": "user", "ai": "assistant"}.get(m[0], m[0])
            out.append({"role": role, "content": m[1]})
        else:
            role = getattr(m, "role", None) or getattr(m, "type", "user")
            out.append({"role": {"human": "user", "ai": "assistant"}.get(role, role),
                        "content": getattr(m, "content", str(m))})
    return out


class LocalChatModel:
    """Chat LLM on the in-process engine (the ChatNVIDIA role)."""

    def __init__(self, service: EngineService, model: str = "local", temperature: float = 0.2,
                 top_p: float = 0.7, max_tokens: int = 1024, stop: Sequence[str] = (),
                 seed: Optional[int] = None, **_ignored):
        self.service = service
        self.model = model
        self.defaults = dict(temperature=temperature, top_p=top_p, max_tokens=max_tokens,
                             stop=list(stop), seed=seed)
        self.tok = service.engine.tok
        self.last_handle: Optional[StreamHandle] = None

    def _params(self, **kw) -> SamplingParams:
        d = dict(self.defaults)
        for k, v in kw.items():
            if v is not None and k in ("temperature", "top_p", "max_tokens", "stop", "seed", "top_k",
                                       "repetition_penalty", "ignore_eos", "stop_token_ids",
                                       "frequency_penalty", "presence_penalty", "beam_width",
                                       "length_penalty", "response_format"):
                d[k] = v.get("type") if k == "response_format" and isinstance(v, dict) else v
        return SamplingParams(**d)

    def _submit(self, messages: Messages, **kw) -> StreamHandle:
        ids = self.service.engine.apply_chat_template(normalize_messages(messages))
        h = self.service.submit(ids, self._params(**kw))
        self.last_handle = h
        return h

    def stream(self, messages: Messages, **kw) -> Iterator[str]:
        h = self._submit(messages, **kw)
        try:
            yield from h
        finally:
            if not h.done.is_set():
                h.cancel()

    def submit(self, messages: Messages, **kw) -> StreamHandle:
        """Queue the request now; stream it later with ``astream(..., handle=h)``."""
        return self._submit(messages, **kw)

    async def astream(self, messages: Messages, coalesce: bool = False, handle: Optional[StreamHandle] = None,
                      **kw):
        """Async token stream straight from the engine's asyncio queue (no worker thread);
        ``coalesce`` joins the deltas that are already queued into one chunk; ``handle``: a
        request already queued by :meth:`submit`."""
        h = handle if handle is not None else self._submit(messages, **kw)
        try:
            async for d in h.aiter(coalesce=coalesce):
                yield d
        finally:
            if not h.done.is_set():
                h.cancel()

    def invoke(self, messages: Messages, **kw) -> str:
        return self._submit(messages, **kw).text()

    __call__ = invoke

    def bind(self, **kw) -> "LocalChatModel":
        m = LocalChatModel(self.service, self.model, **{**self.defaults, **kw})
        return m


class LocalEmbeddings:
    """Embedding client on the in-process encoder (the NVIDIAEmbeddings role)."""

    def __init__(self, engine, model: str = "local", truncate: str = "END", batcher=None):
        self.engine = engine
        self.model = model
        self.truncate = truncate
        self.batcher = batcher

    @property
    def dim(self) -> int:
        return self.engine.dim

    def _embed(self, texts: Sequence[str], input_type: str):
        if self.batcher is not None:
            return self.batcher.embed(list(texts), input_type, self.truncate)
        return self.engine.embed(texts, input_type, self.truncate)

    def embed_query(self, text: str) -> List[float]:
        return self._embed([text], "query")[0].tolist()

    def embed_documents(self, texts: Sequence[str]) -> List[List[float]]:
        return self._embed(texts, "passage").tolist()

    def embed_query_tensor(self, texts: Sequence[str]):
        return self._embed(texts, "query")

    def embed_documents_tensor(self, texts: Sequence[str]):
        return self._embed(texts, "passage")


class LocalReranker:
    """Cross-encoder reranker (the NeMo Retriever reranking role)."""

    def __init__(self, engine, model: str = "local", top_n: int = 4):
        self.engine = engine
        self.model = model
        self.top_n = top_n

    def rank(self, query: str, passages: Sequence[str]) -> List[dict]:
        logits = self.engine.rerank(query, list(passages))
        order = sorted(range(len(logits)), key=lambda i: -logits[i])
        return [{"index": i, "logit": float(logits[i])} for i in order]

    def compress_documents(self, documents, query: str):
        ranks = self.rank(query, [d.page_content for d in documents])
        out = []
        for r in ranks[: self.top_n]:
            d = documents[r["index"]]
            d.metadata = {**d.metadata, "relevance_score": r["logit"]}
            out.append(d)
        return out
