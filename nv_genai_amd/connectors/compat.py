"""Drop-in connector names for code written against the reference.

The reference's chains, notebooks and tools build their clients from
``langchain_nvidia_ai_endpoints`` (``ChatNVIDIA``, ``NVIDIAEmbeddings``, ``NVIDIARerank``:
``RetrievalAugmentedGeneration/common/utils.py:265-316``, ``notebooks/08_RAG_Langchain_with_Local_NIM.ipynb#cell 7``,
``tools/evaluation/rag_evaluator/evaluator.py:110-112``) and wrap embeddings for LlamaIndex
with ``LangchainEmbedding`` (``common/utils.py:136-146``). Switching a script over is an import
change::

    from langchain_nvidia_ai_endpoints import ChatNVIDIA, NVIDIAEmbeddings, NVIDIARerank
    ->  from nv_genai_amd.connectors.compat import ChatNVIDIA, NVIDIAEmbeddings, NVIDIARerank

Same constructor keywords (``model``, ``base_url``, ``nvidia_api_key`` / ``api_key``,
``temperature``, ``top_p``, ``max_tokens``, ``stop``, ``seed``; ``model_type``, ``truncate``;
``top_n``) and the methods those scripts call: ``invoke`` / ``stream`` / ``batch`` / ``bind``
returning message objects with ``.content``; ``embed_query`` / ``embed_documents``;
``compress_documents`` / ``rank``. A ``base_url`` talks to this framework's model server (or
any OpenAI/NIM-compatible endpoint) over HTTP; ``engine=`` (an ``EngineService`` for chat, an
``EmbeddingEngine`` for embeddings / ranking) runs in-process with no HTTP hop. With neither,
``APP_LLM_SERVERURL`` / ``APP_EMBEDDINGS_SERVERURL`` / ``APP_RANKING_SERVERURL`` (the reference's
config names, ``host:port``) or ``http://localhost:8000/v1``.

LlamaIndex-style twins for the ``developer_rag`` path: :class:`NVIDIA` (``complete`` /
``stream_complete`` / ``chat`` / ``stream_chat`` / ``metadata``), :class:`NVIDIAEmbedding` and
:class:`LangchainEmbedding` (``get_query_embedding`` / ``get_text_embedding`` /
``get_text_embedding_batch`` and their ``aget_*`` forms).

``langchain`` / ``llama_index`` are not installed here; these are plain classes with the same
surface, not subclasses of those frameworks' base classes.
"""
from __future__ import annotations

import asyncio
import copy
import os
from dataclasses import dataclass, field
from typing import Any, Iterator, List, Optional, Sequence

from .http import ChatClient, EmbeddingsClient, RerankClient
from .local import LocalChatModel, LocalEmbeddings, LocalReranker, normalize_messages

__all__ = ["AIMessage", "AIMessageChunk", "ChatNVIDIA", "NVIDIAEmbeddings", "NVIDIARerank", "NVIDIA",
           "NVIDIAEmbedding", "LangchainEmbedding", "CompletionResponse", "ChatMessage", "ChatResponse",
           "LLMMetadata"]


def _default_base(env: str) -> str:
    url = os.environ.get(env) or os.environ.get("APP_LLM_SERVERURL") or "localhost:8000"
    return url if url.startswith("http") else f"http://{url}"


def _messages(inp) -> list:
    """LangChain inputs: a string, a PromptValue (``to_messages()``), or a message list."""
    if hasattr(inp, "to_messages"):
        inp = inp.to_messages()
    return normalize_messages(inp)


# ---------------------------------------------------------------------------- LangChain-style
@dataclass
class AIMessage:
    """What ``ChatNVIDIA.invoke`` returns: ``.content`` is the reply text."""
    content: str
    response_metadata: dict = field(default_factory=dict)
    type: str = "ai"

    def __str__(self) -> str:
        return self.content


@dataclass
class AIMessageChunk(AIMessage):
    """A streamed delta; chunks add up to the whole message."""

    def __add__(self, other: "AIMessageChunk") -> "AIMessageChunk":
        return AIMessageChunk(self.content + other.content, {**self.response_metadata, **other.response_metadata})


class ChatNVIDIA:
    """Chat model with the ``langchain_nvidia_ai_endpoints.ChatNVIDIA`` surface."""

    def __init__(self, model: str = "meta/llama3-8b-instruct", base_url: Optional[str] = None,
                 nvidia_api_key: Optional[str] = None, api_key: Optional[str] = None,
                 temperature: float = 0.2, top_p: float = 0.7, max_tokens: int = 1024,
                 stop: Optional[Sequence[str]] = None, seed: Optional[int] = None, engine=None,
                 **kwargs: Any):
        self.model = model
        self.base_url = None if engine is not None else (base_url or _default_base("APP_LLM_SERVERURL"))
        self._kw = dict(temperature=temperature, top_p=top_p, max_tokens=max_tokens,
                        stop=list(stop or ()), seed=seed)
        self._engine = engine
        self._api_key = nvidia_api_key or api_key
        self._extra = kwargs   # further sampling knobs (top_k, repetition_penalty, ...) per call
        if engine is not None:
            self._impl = LocalChatModel(engine, model, **self._kw)
        else:
            self._impl = ChatClient(self.base_url, model, api_key=self._api_key, **self._kw)

    def _call_kw(self, stop, kw) -> dict:
        out = {**self._extra, **kw}
        if stop is not None:
            out["stop"] = list(stop)
        return out

    def invoke(self, input, config: Optional[dict] = None, stop: Optional[Sequence[str]] = None,
               **kwargs) -> AIMessage:
        return AIMessage(self._impl.invoke(_messages(input), **self._call_kw(stop, kwargs)),
                         {"model_name": self.model})

    def stream(self, input, config: Optional[dict] = None, stop: Optional[Sequence[str]] = None,
               **kwargs) -> Iterator[AIMessageChunk]:
        for delta in self._impl.stream(_messages(input), **self._call_kw(stop, kwargs)):
            yield AIMessageChunk(delta)

    def batch(self, inputs: Sequence, config: Optional[dict] = None, **kwargs) -> List[AIMessage]:
        return [self.invoke(i, **kwargs) for i in inputs]

    async def ainvoke(self, input, config: Optional[dict] = None, **kwargs) -> AIMessage:
        return await asyncio.to_thread(self.invoke, input, **kwargs)

    def bind(self, **kwargs) -> "ChatNVIDIA":
        """A copy whose every call also passes ``kwargs`` (e.g. ``stop=[...]``)."""
        other = copy.copy(self)
        other._extra = {**self._extra, **kwargs}
        return other

    __call__ = invoke


class NVIDIAEmbeddings:
    """Embeddings with the ``NVIDIAEmbeddings`` surface. ``model_type`` ("query" / "passage"),
    when given, fixes the input type of both methods, as in the reference's notebooks."""

    def __init__(self, model: str = "snowflake/arctic-embed-l", model_type: Optional[str] = None,
                 truncate: str = "END", base_url: Optional[str] = None,
                 nvidia_api_key: Optional[str] = None, api_key: Optional[str] = None, engine=None,
                 batcher=None, **_ignored):
        if model_type not in (None, "query", "passage"):
            raise ValueError("model_type must be 'query', 'passage' or None")
        self.model, self.model_type, self.truncate = model, model_type, truncate
        if engine is not None:
            self._impl = LocalEmbeddings(engine, model, truncate, batcher)
        else:
            self._impl = EmbeddingsClient(base_url or _default_base("APP_EMBEDDINGS_SERVERURL"), model, truncate,
                                          api_key=nvidia_api_key or api_key)

    def _embed(self, texts: Sequence[str], default: str) -> List[List[float]]:
        v = self._impl._embed(list(texts), self.model_type or default)
        return v.tolist() if hasattr(v, "tolist") else v

    def embed_query(self, text: str) -> List[float]:
        return self._embed([text], "query")[0]

    def embed_documents(self, texts: Sequence[str]) -> List[List[float]]:
        return self._embed(texts, "passage")

    async def aembed_query(self, text: str) -> List[float]:
        return await asyncio.to_thread(self.embed_query, text)

    async def aembed_documents(self, texts: Sequence[str]) -> List[List[float]]:
        return await asyncio.to_thread(self.embed_documents, texts)


class NVIDIARerank:
    """Reranker with the ``NVIDIARerank`` document-compressor surface."""

    def __init__(self, model: str = "nv-rerank-qa-mistral-4b:1", top_n: int = 5,
                 base_url: Optional[str] = None, nvidia_api_key: Optional[str] = None,
                 api_key: Optional[str] = None, engine=None, **_ignored):
        self.model, self.top_n = model, top_n
        if engine is not None:
            self._impl = LocalReranker(engine, model, top_n)
        else:
            self._impl = RerankClient(base_url or _default_base("APP_RANKING_SERVERURL"), model, top_n,
                                      api_key=nvidia_api_key or api_key)

    def rank(self, query: str, passages: Sequence[str]) -> List[dict]:
        return self._impl.rank(query, list(passages))

    def compress_documents(self, documents: Sequence, query: str) -> list:
        """The top ``top_n`` documents (objects with ``page_content`` / ``metadata``) by
        relevance, as copies with ``metadata["relevance_score"]`` set."""
        ranks = self.rank(query, [d.page_content for d in documents])
        out = []
        for r in ranks[: self.top_n]:
            d = copy.copy(documents[r["index"]])
            d.metadata = {**(getattr(d, "metadata", None) or {}), "relevance_score": r["logit"]}
            out.append(d)
        return out


# ---------------------------------------------------------------------------- LlamaIndex-style
@dataclass
class CompletionResponse:
    text: str
    delta: Optional[str] = None


@dataclass
class ChatMessage:
    role: str = "user"
    content: str = ""


@dataclass
class ChatResponse:
    message: ChatMessage
    delta: Optional[str] = None


@dataclass
class LLMMetadata:
    context_window: int = 8192
    num_output: int = 1024
    model_name: str = ""
    is_chat_model: bool = True


class NVIDIA:
    """LLM with the LlamaIndex ``llms.nvidia.NVIDIA`` surface, on the same backends as
    :class:`ChatNVIDIA` (a prompt goes in as one user message)."""

    def __init__(self, model: str = "meta/llama3-8b-instruct", base_url: Optional[str] = None,
                 api_key: Optional[str] = None, temperature: float = 0.2, top_p: float = 0.7,
                 max_tokens: int = 1024, context_window: int = 8192, engine=None, **kwargs):
        self._chat = ChatNVIDIA(model, base_url, api_key=api_key, temperature=temperature, top_p=top_p,
                                max_tokens=max_tokens, engine=engine, **kwargs)
        self.metadata = LLMMetadata(context_window, max_tokens, model, True)

    @staticmethod
    def _msgs(messages: Sequence) -> list:
        return [{"role": getattr(m, "role", "user"), "content": getattr(m, "content", str(m))}
                if not isinstance(m, dict) else m for m in messages]

    def complete(self, prompt: str, **kwargs) -> CompletionResponse:
        return CompletionResponse(self._chat.invoke(prompt, **kwargs).content)

    def stream_complete(self, prompt: str, **kwargs) -> Iterator[CompletionResponse]:
        text = ""
        for ch in self._chat.stream(prompt, **kwargs):
            text += ch.content
            yield CompletionResponse(text, ch.content)

    def chat(self, messages: Sequence, **kwargs) -> ChatResponse:
        return ChatResponse(ChatMessage("assistant", self._chat.invoke(self._msgs(messages), **kwargs).content))

    def stream_chat(self, messages: Sequence, **kwargs) -> Iterator[ChatResponse]:
        text = ""
        for ch in self._chat.stream(self._msgs(messages), **kwargs):
            text += ch.content
            yield ChatResponse(ChatMessage("assistant", text), ch.content)

    async def acomplete(self, prompt: str, **kwargs) -> CompletionResponse:
        return await asyncio.to_thread(self.complete, prompt, **kwargs)


class LangchainEmbedding:
    """LlamaIndex embedding surface over a LangChain-style embeddings object (the reference
    wraps ``NVIDIAEmbeddings`` / ``HuggingFaceEmbeddings`` this way for its LlamaIndex chains)."""

    def __init__(self, lc_embeddings, embed_batch_size: int = 64):
        self.lc = lc_embeddings
        self.embed_batch_size = embed_batch_size

    def get_query_embedding(self, query: str) -> List[float]:
        return self.lc.embed_query(query)

    def get_text_embedding(self, text: str) -> List[float]:
        return self.lc.embed_documents([text])[0]

    def get_text_embedding_batch(self, texts: Sequence[str], **_kw) -> List[List[float]]:
        out: List[List[float]] = []
        for i in range(0, len(texts), self.embed_batch_size):
            out += self.lc.embed_documents(list(texts[i:i + self.embed_batch_size]))
        return out

    async def aget_query_embedding(self, query: str) -> List[float]:
        return await asyncio.to_thread(self.get_query_embedding, query)

    async def aget_text_embedding(self, text: str) -> List[float]:
        return await asyncio.to_thread(self.get_text_embedding, text)


class NVIDIAEmbedding(LangchainEmbedding):
    """LlamaIndex ``embeddings.nvidia.NVIDIAEmbedding`` surface."""

    def __init__(self, model: str = "snowflake/arctic-embed-l", truncate: str = "END",
                 base_url: Optional[str] = None, api_key: Optional[str] = None, engine=None,
                 embed_batch_size: int = 64, **kwargs):
        super().__init__(NVIDIAEmbeddings(model, None, truncate, base_url, api_key=api_key, engine=engine,
                                          **kwargs), embed_batch_size)
