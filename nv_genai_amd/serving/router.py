"""Request router over data-parallel model-server replicas (NIM
``num_instances``, ``--scale ingest-worker=N``): one model server per GPU (8B + encoder fit a
single MI355X many times over), the router sends each request to the replica with the fewest
in-flight requests and streams the response through unchanged.

``python -m nv_genai_amd.serving.router --backends http://gpu0:8000,http://gpu1:8001 --port 8080``
"""
from __future__ import annotations

import argparse
import asyncio
import contextlib
import threading
from typing import List

import httpx
from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, Response, StreamingResponse


class Router:
    def __init__(self, backends: List[str]):
        self.backends = [b.rstrip("/") for b in backends]
        self.inflight = {b: 0 for b in self.backends}
        self.healthy = {b: True for b in self.backends}
        self.lock = threading.Lock()

    def pick(self) -> str:
        with self.lock:
            cands = [b for b in self.backends if self.healthy[b]] or self.backends
            b = min(cands, key=lambda x: self.inflight[x])
            self.inflight[b] += 1
            return b

    def done(self, b: str):
        with self.lock:
            self.inflight[b] -= 1


def create_router(backends: List[str], timeout: float = 600.0) -> FastAPI:
    r = Router(backends)
    client = httpx.AsyncClient(timeout=timeout)

    @contextlib.asynccontextmanager
    async def lifespan(app):
        task = asyncio.create_task(health_loop())
        yield
        task.cancel()

    app = FastAPI(title="nv_genai_amd router", lifespan=lifespan)
    app.state.router = r

    @app.api_route("/v1/{path:path}", methods=["GET", "POST"])
    async def proxy(path: str, request: Request):
        body = await request.body()
        if request.method == "GET" and path in ("models", "health/ready", "health/live"):
            b = r.backends[0]
            resp = await client.get(f"{b}/v1/{path}")
            return Response(resp.content, resp.status_code, media_type=resp.headers.get("content-type"))
        b = r.pick()
        stream = b'"stream": true' in body or b'"stream":true' in body
        headers = {"content-type": request.headers.get("content-type", "application/json")}
        if "traceparent" in request.headers:
            headers["traceparent"] = request.headers["traceparent"]
        if not stream:
            try:
                resp = await client.request(request.method, f"{b}/v1/{path}", content=body, headers=headers)
                return Response(resp.content, resp.status_code, media_type=resp.headers.get("content-type"))
            except httpx.HTTPError as e:
                r.healthy[b] = False
                return JSONResponse({"error": f"backend {b} failed: {e}"}, status_code=502)
            finally:
                r.done(b)

        async def gen():
            try:
                async with client.stream(request.method, f"{b}/v1/{path}", content=body, headers=headers) as resp:
                    async for chunk in resp.aiter_raw():
                        yield chunk
            finally:
                r.done(b)

        return StreamingResponse(gen(), media_type="text/event-stream")

    @app.get("/router/status")
    def status():
        return {"backends": r.backends, "inflight": r.inflight, "healthy": r.healthy}

    async def health_loop():
        while True:
            for b in r.backends:
                try:
                    resp = await client.get(f"{b}/v1/health/ready", timeout=5)
                    r.healthy[b] = resp.status_code == 200
                except httpx.HTTPError:
                    r.healthy[b] = False
            await asyncio.sleep(5)

    return app


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--backends", required=True)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8080)
    args = ap.parse_args(argv)
    import uvicorn

    uvicorn.run(create_router(args.backends.split(",")), host=args.host, port=args.port)


if __name__ == "__main__":
    main()
