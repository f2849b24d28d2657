"""HTTP connectors speaking the OpenAI / NIM wire protocol (SURVEY.md §2.B N1-N3 contracts):

* :class:`ChatClient`  — ``POST {base}/chat/completions`` (``stream=true`` -> SSE
  ``data: {...}`` chunks terminated by ``data: [DONE]``), temperature / top_p / max_tokens /
  stop / seed forwarded (RetrievalAugmentedGeneration/common/utils.py:265-290);
* :class:`EmbeddingsClient` — ``POST {base}/embeddings`` with ``input_type`` query|passage and
  ``truncate`` (experimental/fm-asr-streaming-rag/chain-server/common.py:64-101);
* :class:`RerankClient` — ``POST {base}/ranking`` ``{query:{text}, passages:[{text}]}`` ->
  ``rankings[{index, logit}]`` (experimental/fm-asr-streaming-rag/chain-server/retriever.py:287-306).

They work against this framework's model server and against any OpenAI-compatible endpoint.
"""
from __future__ import annotations

import json
import os
import threading
from typing import Iterator, List, Optional, Sequence

import requests

from .local import Messages, normalize_messages


_TLS = threading.local()


def _session() -> requests.Session:
    """A keep-alive ``requests.Session`` per thread (Sessions are not thread-safe): the vector
    store's query batcher embeds every retrieval batch over HTTP in the split topology, and a
    fresh TCP connection per call showed in its profile (profiles/r5_http/)."""
    s = getattr(_TLS, "s", None)
    if s is None:
        s = _TLS.s = requests.Session()
    return s


def _base(url: str) -> str:
    url = url.rstrip("/")
    if not url.startswith("http"):
        url = "http://" + url
    if not url.endswith("/v1"):
        url += "/v1"
    return url


def _headers(api_key: Optional[str]):
    h = {"Content-Type": "application/json", "Accept": "application/json"}
    key = api_key or os.environ.get("NVIDIA_API_KEY") or os.environ.get("OPENAI_API_KEY")
    if key:
        h["Authorization"] = f"Bearer {key}"
    return h


class ChatClient:
    def __init__(self, base_url: str, model: str = "meta/llama3-8b-instruct",
                 temperature: float = 0.2, top_p: float = 0.7, max_tokens: int = 1024,
                 stop: Sequence[str] = (), seed: Optional[int] = None,
                 api_key: Optional[str] = None, timeout: float = 600.0, headers: Optional[dict] = None):
        self.base = _base(base_url)
        self.model = model
        self.defaults = dict(temperature=temperature, top_p=top_p, max_tokens=max_tokens,
                             stop=list(stop), seed=seed)
        self.api_key = api_key
        self.timeout = timeout
        self.extra_headers = headers or {}

    def _body(self, messages: Messages, stream: bool, **kw) -> dict:
        b = {"model": self.model, "messages": normalize_messages(messages), "stream": stream}
        for k, v in {**self.defaults, **{k: v for k, v in kw.items() if v is not None}}.items():
            if v is None or (k == "stop" and not v):
                continue
            b[k] = v
        return b

    def stream(self, messages: Messages, **kw) -> Iterator[str]:
        with _session().post(f"{self.base}/chat/completions", json=self._body(messages, True, **kw),
                           headers={**_headers(self.api_key), **self.extra_headers},
                           stream=True, timeout=self.timeout) as r:
            r.raise_for_status()
            for line in r.iter_lines(decode_unicode=True):
                if not line or not line.startswith("data:"):
                    continue
                payload = line[5:].strip()
                if payload == "[DONE]":
                    break
                chunk = json.loads(payload)
                for ch in chunk.get("choices", []):
                    delta = ch.get("delta", {}).get("content")
                    if delta:
                        yield delta

    async def astream(self, messages: Messages, coalesce: bool = False, handle=None, **kw):
        """The same SSE stream on the caller's event loop (one pooled aiohttp session per
        loop): an async server forwards an upstream model server's tokens without parking a
        thread per open stream. ``coalesce`` joins the deltas of frames that arrived together.

        aiohttp, not httpx, on this path: a chain server in front of a model server relays one
        frame per token per stream, and httpx's anyio transport re-registers the socket with
        the selector on every read (two epoll_ctl calls per token) and looks for sniffio on
        every request (profiles/r5_http/: the chain server's event loop was the split
        topology's bottleneck); aiohttp's C parser hands over whatever bytes arrived."""
        body = self._body(messages, True, **kw)
        url = f"{self.base}/chat/completions"
        headers = {**_headers(self.api_key), **self.extra_headers}
        session = _aiohttp_session()
        if session is None:   # no aiohttp: httpx
            async for d in self._astream_httpx(url, body, headers, coalesce):
                yield d
            return
        async with session.post(url, json=body, headers=headers, timeout=_aiohttp_timeout(self.timeout)) as r:
            if r.status != 200:
                text = await r.text()
                raise RuntimeError(f"chat/completions returned {r.status}: {text[:200]}")
            carry = [b""]
            while True:
                chunk = await r.content.readany()
                if not chunk:
                    return
                parts, done = _sse_deltas(carry, chunk)
                if parts:
                    if coalesce:
                        yield "".join(parts)
                    else:
                        for p in parts:
                            yield p
                if done:
                    return

    async def _astream_httpx(self, url: str, body: dict, headers: dict, coalesce: bool):
        client = _async_client(self.timeout)
        async with client.stream("POST", url, json=body, headers=headers) as r:
            if r.status_code != 200:
                await r.aread()
                raise RuntimeError(f"chat/completions returned {r.status_code}: {r.text[:200]}")
            carry = [b""]
            async for chunk in r.aiter_bytes():
                parts, done = _sse_deltas(carry, chunk)
                if parts:
                    if coalesce:
                        yield "".join(parts)
                    else:
                        for p in parts:
                            yield p
                if done:
                    return

    def invoke(self, messages: Messages, **kw) -> str:
        r = _session().post(f"{self.base}/chat/completions", json=self._body(messages, False, **kw),
                          headers={**_headers(self.api_key), **self.extra_headers}, timeout=self.timeout)
        r.raise_for_status()
        return r.json()["choices"][0]["message"]["content"]

    __call__ = invoke


def _sse_lines(carry: list, text: str):
    """Complete ``data:`` payloads in a text chunk of an SSE stream; a partial last line is
    kept in ``carry[0]`` (one per stream) until the next chunk completes it."""
    *lines, carry[0] = (carry[0] + text).split("\n")
    for line in lines:
        if line.startswith("data:"):
            yield line[5:].strip()


def _sse_deltas(carry: list, chunk: bytes):
    """(content deltas, saw [DONE]) of the complete ``data:`` lines in a byte chunk of an
    OpenAI chat stream; the partial last line stays in ``carry[0]``. Lines are split as bytes,
    so a UTF-8 character cut across two chunks is decoded whole."""
    *lines, carry[0] = (carry[0] + chunk).split(b"\n")
    parts = []
    for line in lines:
        if not line.startswith(b"data:"):
            continue
        payload = line[5:].strip()
        if payload == b"[DONE]":
            return parts, True
        for ch in json.loads(payload).get("choices", []):
            delta = ch.get("delta", {}).get("content")
            if delta:
                parts.append(delta)
    return parts, False


_ASYNC_CLIENTS = {}
_AIOHTTP_SESSIONS = {}


def _aiohttp_timeout(timeout: float):
    """Per-request aiohttp timeout with the same meaning as the requests / httpx paths: the
    limit applies to connecting and to each read, never to the whole stream (a long generation
    relayed token by token must not be cut off at ``timeout`` seconds)."""
    import aiohttp

    return aiohttp.ClientTimeout(total=None, sock_connect=timeout, sock_read=timeout)


def _aiohttp_session():
    """One pooled aiohttp.ClientSession per event loop (no connection cap: every open stream
    holds one), or None without aiohttp. Timeouts are per request (:func:`_aiohttp_timeout`),
    so clients with different timeouts can share the session."""
    import asyncio

    try:
        import aiohttp
    except ImportError:   # pragma: no cover - aiohttp ships in the image
        return None
    loop = asyncio.get_running_loop()
    s = _AIOHTTP_SESSIONS.get(id(loop))
    if s is None or s[0] is not loop or s[1].closed:
        s = (loop, aiohttp.ClientSession(connector=aiohttp.TCPConnector(limit=0, keepalive_timeout=60),
                                         timeout=aiohttp.ClientTimeout(total=None)))
        _AIOHTTP_SESSIONS[id(loop)] = s
    return s[1]


async def aclose_clients() -> None:
    """Close this event loop's pooled aiohttp session / httpx client (server shutdown)."""
    import asyncio

    key = id(asyncio.get_running_loop())
    s = _AIOHTTP_SESSIONS.pop(key, None)
    if s is not None and not s[1].closed:
        await s[1].close()
    c = _ASYNC_CLIENTS.pop(key, None)
    if c is not None:
        await c[1].aclose()


def _async_client(timeout: float):
    """One pooled httpx.AsyncClient per event loop (connections are reused across streams)."""
    import asyncio
    import importlib.util
    import sys

    import httpx

    if "sniffio" not in sys.modules and importlib.util.find_spec("sniffio") is None:
        # httpcore tries `import sniffio` on every request; absent, each failed import walks
        # sys.path. A None entry makes the import fail at once (httpcore then assumes asyncio)
        sys.modules["sniffio"] = None
    loop = asyncio.get_running_loop()
    c = _ASYNC_CLIENTS.get(id(loop))
    if c is None or c[0] is not loop:
        c = (loop, httpx.AsyncClient(timeout=httpx.Timeout(timeout),
                                     limits=httpx.Limits(max_connections=4096, max_keepalive_connections=1024)))
        _ASYNC_CLIENTS[id(loop)] = c
    return c[1]


class EmbeddingsClient:
    def __init__(self, base_url: str, model: str = "snowflake/arctic-embed-l", truncate: str = "END",
                 api_key: Optional[str] = None, timeout: float = 120.0, batch_size: int = 256):
        self.base = _base(base_url)
        self.model = model
        self.truncate = truncate
        self.api_key = api_key
        self.timeout = timeout
        self.batch_size = batch_size

    def _embed(self, texts: Sequence[str], input_type: str) -> List[List[float]]:
        out: List[List[float]] = []
        for i in range(0, len(texts), self.batch_size):
            body = {"input": list(texts[i:i + self.batch_size]), "model": self.model,
                    "input_type": input_type, "truncate": self.truncate,
                    "encoding_format": "float"}
            r = _session().post(f"{self.base}/embeddings", json=body, headers=_headers(self.api_key),
                              timeout=self.timeout)
            r.raise_for_status()
            data = sorted(r.json()["data"], key=lambda d: d["index"])
            out += [d["embedding"] for d in data]
        return out

    def embed_query(self, text: str) -> List[float]:
        return self._embed([text], "query")[0]

    def embed_query_tensor(self, texts: Sequence[str]):
        """[n, dim] fp32 tensor of a batch of queries in ONE request (the vector store's query
        batcher coalesces concurrent searches), base64 little-endian fp32 on the wire."""
        import base64

        import numpy as np
        import torch

        out = []
        for i in range(0, len(texts), self.batch_size):
            body = {"input": list(texts[i:i + self.batch_size]), "model": self.model, "input_type": "query",
                    "truncate": self.truncate, "encoding_format": "base64"}
            r = _session().post(f"{self.base}/embeddings", json=body, headers=_headers(self.api_key),
                              timeout=self.timeout)
            r.raise_for_status()
            for d in sorted(r.json()["data"], key=lambda d: d["index"]):
                e = d["embedding"]
                out.append(np.frombuffer(base64.b64decode(e), dtype="<f4") if isinstance(e, str)
                           else np.asarray(e, dtype=np.float32))
        return torch.from_numpy(np.stack(out).astype(np.float32)) if out else torch.zeros(0, 0)

    def embed_documents(self, texts: Sequence[str]) -> List[List[float]]:
        return self._embed(texts, "passage")


class RerankClient:
    def __init__(self, base_url: str, model: str = "nv-rerank-qa-mistral-4b:1", top_n: int = 4,
                 api_key: Optional[str] = None, timeout: float = 120.0):
        self.base = _base(base_url)
        self.model = model
        self.top_n = top_n
        self.api_key = api_key
        self.timeout = timeout

    def rank(self, query: str, passages: Sequence[str]) -> List[dict]:
        body = {"model": self.model, "query": {"text": query},
                "passages": [{"text": p} for p in passages]}
        r = _session().post(f"{self.base}/ranking", json=body, headers=_headers(self.api_key),
                          timeout=self.timeout)
        r.raise_for_status()
        return r.json()["rankings"]
