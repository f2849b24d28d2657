"""Response-caching reverse proxy for LLM / embedding APIs (SURVEY.md §2.G "Response
caching"; reference: experimental/event-driven-rag-cve-analysis/nginx — ``proxy_cache`` keyed
on method + URI + request body for the OpenAI-style POSTs, 14-day validity, stale responses
served when the upstream errors).

Identical requests (same method, path, query and body bytes) are answered from an on-disk
SQLite cache; streamed (SSE) responses are passed through chunk by chunk and stored once
complete. ``X-Cache-Status`` is MISS / HIT / STALE like nginx's ``$upstream_cache_status``.

``python -m nv_genai_amd.serving.cache_proxy --upstream http://localhost:8000 --port 8080``
"""
from __future__ import annotations

import argparse
import hashlib
import sqlite3
import threading
import time
from typing import Optional

import httpx
from fastapi import FastAPI, Request
from fastapi.responses import Response, StreamingResponse

DAY = 86400.0


class ResponseCache:
    def __init__(self, path: str = ":memory:", ttl: float = 14 * DAY):
        self.db = sqlite3.connect(path, check_same_thread=False)
        self.lock = threading.Lock()
        self.ttl = ttl
        with self.lock:
            self.db.execute("CREATE TABLE IF NOT EXISTS cache (k TEXT PRIMARY KEY, status INTEGER, ctype TEXT, "
                            "body BLOB, t REAL)")
            self.db.commit()

    @staticmethod
    def key(method: str, uri: str, body: bytes) -> str:
        return hashlib.sha256(method.encode() + b" " + uri.encode() + b"\n" + body).hexdigest()

    def get(self, k: str):
        with self.lock:
            r = self.db.execute("SELECT status, ctype, body, t FROM cache WHERE k = ?", (k,)).fetchone()
        if r is None:
            return None
        status, ctype, body, t = r
        return status, ctype, body, (time.time() - t) <= self.ttl

    def put(self, k: str, status: int, ctype: str, body: bytes):
        with self.lock:
            self.db.execute("INSERT OR REPLACE INTO cache VALUES (?, ?, ?, ?, ?)", (k, status, ctype, body, time.time()))
            self.db.commit()


def create_cache_proxy(upstream: str, cache: Optional[ResponseCache] = None, timeout: float = 600.0,
                       transport: Optional[httpx.AsyncBaseTransport] = None) -> FastAPI:
    app = FastAPI(title="nv_genai_amd response cache")
    cache = cache or ResponseCache()
    client = httpx.AsyncClient(base_url=upstream.rstrip("/"), timeout=timeout, transport=transport)
    app.state.cache = cache

    @app.api_route("/{path:path}", methods=["GET", "POST"])
    async def proxy(path: str, request: Request):
        body = await request.body()
        uri = "/" + path + (("?" + request.url.query) if request.url.query else "")
        k = ResponseCache.key(request.method, uri, body)
        hit = cache.get(k) if request.method == "POST" else None
        if hit is not None and hit[3]:
            return Response(hit[2], hit[0], media_type=hit[1], headers={"X-Cache-Status": "HIT"})
        headers = {h: v for h, v in request.headers.items() if h.lower() in ("content-type", "authorization",
                                                                              "accept", "traceparent")}
        try:
            req = client.build_request(request.method, uri, content=body, headers=headers)
            resp = await client.send(req, stream=True)
        except httpx.HTTPError:
            if hit is not None:
                return Response(hit[2], hit[0], media_type=hit[1], headers={"X-Cache-Status": "STALE"})
            return Response(b'{"error": "upstream unavailable"}', 502, media_type="application/json")
        ctype = resp.headers.get("content-type", "application/octet-stream")
        if resp.status_code >= 500 and hit is not None:
            await resp.aclose()
            return Response(hit[2], hit[0], media_type=hit[1], headers={"X-Cache-Status": "STALE"})
        cacheable = request.method == "POST" and resp.status_code == 200

        async def gen():
            buf = bytearray()
            try:
                async for chunk in resp.aiter_bytes():
                    buf.extend(chunk)
                    yield chunk
            finally:
                await resp.aclose()
            if cacheable:
                cache.put(k, resp.status_code, ctype, bytes(buf))

        return StreamingResponse(gen(), status_code=resp.status_code, media_type=ctype,
                                 headers={"X-Cache-Status": "MISS"})

    return app


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--upstream", required=True)
    ap.add_argument("--cache", default="response_cache.sqlite")
    ap.add_argument("--ttl-days", type=float, default=14.0)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8080)
    a = ap.parse_args(argv)
    import uvicorn

    uvicorn.run(create_cache_proxy(a.upstream, ResponseCache(a.cache, a.ttl_days * DAY)), host=a.host, port=a.port)


if __name__ == "__main__":
    main()
