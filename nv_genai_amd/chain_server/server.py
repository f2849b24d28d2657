"""Chain server: the reference's REST API, byte-compatible (SURVEY.md §2.A C1, §3.2;
RetrievalAugmentedGeneration/common/server.py:44-427, docs/api_reference/openapi_schema.json).

Routes: ``GET /health``, ``POST /documents`` (multipart upload -> ingest), ``GET /documents``,
``DELETE /documents?filename=``, ``POST /generate`` (SSE), ``POST /search``.
Wire format of /generate: ``data: <ChainResponse JSON>\\n\\n`` per chunk, a final chunk with
empty content and ``finish_reason: "[DONE]"``; on failure HTTP 500 with one error chunk.
Request limits are the reference's pydantic constraints; every user string is HTML-sanitised.

Additions (MI355X framework): ``GET /health/ready`` (engines loaded, not stuck) and
``GET /metrics`` (Prometheus text: requests, latency, TTFT, engine/KV state).

Run: ``uvicorn nv_genai_amd.chain_server.server:app --port 8081`` with ``EXAMPLE_NAME``
(package example, default ``developer_rag``) or ``EXAMPLE_PATH`` (a directory of .py files,
like the reference's ``RetrievalAugmentedGeneration/example``).
"""
from __future__ import annotations

import asyncio
import contextlib
import importlib
import json
import importlib.util
import logging
import os
import time
from inspect import getmembers, isclass
from pathlib import Path
from typing import Any, Dict, List
from uuid import uuid4

from fastapi import FastAPI, Request
from fastapi.encoders import jsonable_encoder
from fastapi.exceptions import RequestValidationError
from fastapi.middleware.cors import CORSMiddleware
from fastapi.responses import JSONResponse, PlainTextResponse, StreamingResponse
from pydantic import BaseModel, Field, constr, field_validator
from starlette.background import BackgroundTask
from starlette.concurrency import run_in_threadpool
from starlette.status import HTTP_422_UNPROCESSABLE_ENTITY

from ..observability.metrics import METRICS
from ..observability.tracing import get_tracer
from .multipart import parse_multipart
from .sanitize import clean

logging.basicConfig(level=os.environ.get("LOGLEVEL", "INFO").upper())
logger = logging.getLogger(__name__)

@contextlib.asynccontextmanager
async def _lifespan(_app):
    from ..observability.sampler import start_from_env

    start_from_env("chain")   # NGA_PY_SAMPLE_OUT: stack-sample this process (diagnostics)
    import_example()
    yield
    from ..connectors.http import aclose_clients

    await aclose_clients()   # pooled upstream connections (split topology)


app = FastAPI(title="nv_genai_amd chain server", lifespan=_lifespan)
app.add_middleware(CORSMiddleware, allow_origins=["*"], allow_credentials=False,
                   allow_methods=["*"], allow_headers=["*"])
tracer = get_tracer("chain-server")
UPLOAD_DIR = os.environ.get("UPLOAD_DIR", "/tmp-data/uploaded_files")


class Message(BaseModel):
    role: str = Field(default="user", max_length=256, pattern=r"[\s\S]*",
                      description="Role for a message AI, User and System")
    content: str = Field(default="I am going to Paris, what should I see?", max_length=131072,
                         pattern=r"[\s\S]*", description="The input query/prompt to the pipeline.")

    @field_validator("role")
    @classmethod
    def validate_role(cls, v):
        v = clean(v)
        if v.lower() not in {"user", "assistant", "system"}:
            raise ValueError("Role must be one of 'user', 'assistant', or 'system'")
        return v.lower()

    @field_validator("content")
    @classmethod
    def sanitize_content(cls, v):
        return clean(v)


class Prompt(BaseModel):
    messages: List[Message] = Field(..., max_length=50000)
    use_knowledge_base: bool = Field(..., description="Whether to use a knowledge base")
    temperature: float = Field(0.2, ge=0.1, le=1.0)
    top_p: float = Field(0.7, ge=0.1, le=1.0)
    max_tokens: int = Field(1024, ge=0, le=1024)
    stop: List[constr(max_length=256, pattern=r"[\s\S]*")] = Field(default=[], max_length=256)

    @field_validator("use_knowledge_base", mode="before")
    @classmethod
    def sanitize_use_kb(cls, v):
        v = clean(str(v))
        try:
            return {"True": True, "False": False, "true": True, "false": False}[v]
        except KeyError:
            raise ValueError("use_knowledge_base must be a boolean value")


class ChainResponseChoices(BaseModel):
    index: int = Field(default=0, ge=0, le=256)
    message: Message = Field(default=Message(role="assistant", content=""))
    finish_reason: str = Field(default="", max_length=4096, pattern=r"[\s\S]*")


class ChainResponse(BaseModel):
    id: str = Field(default="", max_length=100000, pattern=r"[\s\S]*")
    choices: List[ChainResponseChoices] = Field(default=[], max_length=256)


class DocumentSearch(BaseModel):
    query: str = Field(default="", max_length=131072, pattern=r"[\s\S]*")
    top_k: int = Field(default=4, ge=0, le=25)


class DocumentChunk(BaseModel):
    content: str = Field(default="", max_length=131072, pattern=r"[\s\S]*")
    filename: str = Field(default="", max_length=4096, pattern=r"[\s\S]*")
    score: float = Field(...)


class DocumentSearchResponse(BaseModel):
    chunks: List[DocumentChunk] = Field(..., max_length=256)


class DocumentsResponse(BaseModel):
    documents: List[constr(max_length=131072, pattern=r"[\s\S]*")] = Field(default=[], max_length=1000000)


class HealthResponse(BaseModel):
    message: str = Field(default="", max_length=4096, pattern=r"[\s\S]*")


# ---------------------------------------------------------------------------- discovery
def _find_example_class(module):
    for name, cls in getmembers(module, isclass):
        if name == "BaseExample":
            continue
        if {"ingest_docs", "llm_chain", "rag_chain"}.issubset(set(dir(cls))):
            return cls
    return None


def load_example():
    path = os.environ.get("EXAMPLE_PATH")
    if path:
        for root, _dirs, files in os.walk(path):
            for f in sorted(files):
                if not f.endswith(".py"):
                    continue
                spec = importlib.util.spec_from_file_location("example", os.path.join(root, f))
                mod = importlib.util.module_from_spec(spec)
                spec.loader.exec_module(mod)
                cls = _find_example_class(mod)
                if cls is not None:
                    cls()  # instantiate once as a check, like the reference
                    return cls
        raise NotImplementedError(f"Could not find a valid example class in {path}")
    name = os.environ.get("EXAMPLE_NAME", "developer_rag")
    mod = importlib.import_module(f"nv_genai_amd.examples.{name}.chains")
    cls = _find_example_class(mod)
    if cls is None:
        raise NotImplementedError(f"Could not find a valid example class in example {name}")
    cls()
    return cls


def import_example() -> None:
    """Start-up (the app's lifespan): thread pool sizing, example discovery, engines."""
    # every open /generate stream parks a worker thread on its token queue between chunks
    # (sync example generators): size the pool for the serving concurrency, not anyio's 40
    import anyio.to_thread

    anyio.to_thread.current_default_thread_limiter().total_tokens = int(os.environ.get("APP_THREADPOOL", "2048"))
    # GIL hand-off interval (tuning knob; measured: 0.2 / 0.5 ms did not beat CPython's 5 ms
    # default on the REST RAG benchmark, profiles/r4_http/)
    if os.environ.get("APP_GIL_SWITCH_US"):
        import sys

        sys.setswitchinterval(float(os.environ["APP_GIL_SWITCH_US"]) * 1e-6)
    if getattr(app, "example", None) is None:
        app.example = load_example()
    # in-process engines are built (weights, KV cache, decode hipGraphs) before traffic arrives
    from . import utils

    cfg = utils.get_config()
    if cfg.llm.model_engine == "local" and os.environ.get("APP_LAZY_ENGINES", "0") != "1":
        utils.get_llm_service()


@app.exception_handler(RequestValidationError)
async def request_validation_exception_handler(request: Request, exc: RequestValidationError) -> JSONResponse:
    return JSONResponse(status_code=HTTP_422_UNPROCESSABLE_ENTITY,
                        content={"detail": jsonable_encoder(exc.errors(), exclude={"input", "ctx", "url"})})


def _traceparent(request: Request):
    return request.headers.get("traceparent")


# ---------------------------------------------------------------------------- routes
@app.get("/health", response_model=HealthResponse)
def health_check():
    """Returns 200 when the service is up (does not check downstream services)."""
    return HealthResponse(message="Service is up.")


@app.get("/health/ready")
def ready():
    from . import utils

    svc = utils._RUNTIME.get("llm_service")
    ok = getattr(app, "example", None) is not None and (svc is None or svc.healthy())
    return JSONResponse({"ready": ok}, status_code=200 if ok else 503)


@app.get("/metrics")
def metrics():
    from . import utils

    svc = utils._RUNTIME.get("llm_service")
    extra = svc.metrics() if svc is not None else {}
    return PlainTextResponse(METRICS.render(extra, prefix="chain_server"), media_type="text/plain; version=0.0.4")


@app.post("/documents")
async def upload_document(request: Request) -> JSONResponse:
    try:
        parts = parse_multipart(await request.body(), request.headers.get("content-type", ""))
    except ValueError:
        parts = {}
    if "file" not in parts:
        return JSONResponse(status_code=HTTP_422_UNPROCESSABLE_ENTITY, content={"detail": [
            {"type": "missing", "loc": ["body", "file"], "msg": "Field required"}]})
    filename, data = parts["file"]
    if not filename:
        return JSONResponse(content={"message": "No files provided"}, status_code=200)
    with tracer.span("POST /documents", {"filename": filename}, _traceparent(request)):
        try:
            upload_file = os.path.basename(filename)
            if not upload_file:
                raise RuntimeError("Error parsing uploaded filename.")
            Path(UPLOAD_DIR).mkdir(parents=True, exist_ok=True)
            file_path = os.path.join(UPLOAD_DIR, upload_file)
            with open(file_path, "wb") as f:
                f.write(data)
            t0 = time.perf_counter()
            await asyncio.to_thread(app.example().ingest_docs, file_path, upload_file)
            METRICS.observe("ingest_seconds", time.perf_counter() - t0)
            return JSONResponse(content={"message": "File uploaded successfully"}, status_code=200)
        except Exception as e:  # noqa: BLE001
            logger.error("Error from POST /documents endpoint. Ingestion of file: %s failed with error: %s",
                         filename, e)
            return JSONResponse(content={"message": str(e)}, status_code=500)


_MARK = "\u2063SPLICE\u2063"


def _frame_parts(resp_id: str):
    """SSE frame of one ChainResponse chunk split around its content field."""
    r = ChainResponse(id=resp_id, choices=[ChainResponseChoices(
        index=0, message=Message(role="assistant", content=_MARK))])
    head, tail = ("data: " + r.model_dump_json() + "\n\n").split(_MARK)
    return head, tail


def _error_stream(msg: str) -> StreamingResponse:
    resp = ChainResponse(choices=[ChainResponseChoices(index=0, message=Message(role="assistant", content=msg),
                                                       finish_reason="[DONE]")])
    return StreamingResponse(iter(["data: " + resp.model_dump_json() + "\n\n"]),
                             media_type="text/event-stream", status_code=500)


@app.post("/generate", response_model=ChainResponse)
async def generate_answer(request: Request, prompt: Prompt) -> StreamingResponse:
    chat_history = prompt.messages
    last_user_message = next((m.content for m in reversed(chat_history) if m.role == "user"), None)
    for i in reversed(range(len(chat_history))):
        if chat_history[i].role == "user":
            del chat_history[i]
            break
    llm_settings = {k: v for k, v in vars(prompt).items() if k not in ("messages", "use_knowledge_base")}
    span = tracer.start("POST /generate", attributes={"use_knowledge_base": prompt.use_knowledge_base},
                        traceparent=_traceparent(request))
    t_start = time.perf_counter()
    METRICS.inc("generate_requests_total")
    try:
        example = app.example()
        # the chain's synchronous part (retrieval, prompt assembly) runs on a worker thread:
        # on the event loop it would serialise every request's retrieval and stall all streams,
        # and concurrent requests' searches could never share a batch (VectorStore batcher)
        chain = example.rag_chain if prompt.use_knowledge_base else example.llm_chain

        def run_chain():
            t0 = time.perf_counter()
            g = chain(query=last_user_message, chat_history=chat_history, **llm_settings)
            if hasattr(g, "prepare"):
                t1 = time.perf_counter()
                g.prepare()      # prompt tokenised + queued on the engine from this thread
                METRICS.observe("prepare_seconds", time.perf_counter() - t1)
            METRICS.observe("chain_seconds", time.perf_counter() - t0)
            return g

        # anyio's pool (limiter raised to APP_THREADPOOL at startup), not asyncio's default
        # executor of min(32, cpus + 4) threads: every concurrent request's retrieval must be
        # in flight at once for the vector store's batcher to coalesce them
        generator = await run_in_threadpool(run_chain)
        METRICS.observe("chain_wait_seconds", time.perf_counter() - t_start)
    except Exception as e:  # noqa: BLE001
        logger.error("Error from /generate endpoint. Error details: %s", e)
        METRICS.inc("generate_errors_total")
        tracer.end(span)
        return _error_stream("Error from chain server. Please check chain-server logs for more details.")

    def response_generator():
        resp_id = str(uuid4())
        first = True
        try:
            if generator:
                for chunk in generator:
                    if first:
                        METRICS.observe("ttft_seconds", time.perf_counter() - t_start)
                        first = False
                    r = ChainResponse(id=resp_id, choices=[ChainResponseChoices(
                        index=0, message=Message(role="assistant", content=chunk))])
                    yield "data: " + r.model_dump_json() + "\n\n"
                r = ChainResponse(id=resp_id, choices=[ChainResponseChoices(finish_reason="[DONE]")])
                yield "data: " + r.model_dump_json() + "\n\n"
            else:
                yield "data: " + ChainResponse().model_dump_json() + "\n\n"
        except Exception as e:  # noqa: BLE001 - mid-stream failure: close with an error chunk
            logger.error("Error while streaming /generate: %s", e)
            METRICS.inc("generate_errors_total")
            r = ChainResponse(id=resp_id, choices=[ChainResponseChoices(
                index=0, message=Message(role="assistant",
                                         content="Error from chain server. Please check chain-server logs for more details."),
                finish_reason="[DONE]")])
            yield "data: " + r.model_dump_json() + "\n\n"
        finally:
            METRICS.observe("generate_seconds", time.perf_counter() - t_start)
            tracer.end(span)

    async def response_agen():
        """Same frames, fed from the engine's asyncio queue (LLMStream over a local engine).
        Frames are the ChainResponse JSON with the sanitised chunk spliced in (byte-identical
        to model_dump_json, without a pydantic round trip per token)."""
        resp_id = str(uuid4())
        head, tail = _frame_parts(resp_id)
        first = True
        try:
            async for chunk in generator:
                if first:
                    METRICS.observe("ttft_seconds", time.perf_counter() - t_start)
                    first = False
                yield head + json.dumps(clean(chunk), ensure_ascii=False)[1:-1] + tail
            r = ChainResponse(id=resp_id, choices=[ChainResponseChoices(finish_reason="[DONE]")])
            yield "data: " + r.model_dump_json() + "\n\n"
        except Exception as e:  # noqa: BLE001
            logger.error("Error while streaming /generate: %s", e)
            METRICS.inc("generate_errors_total")
            r = ChainResponse(id=resp_id, choices=[ChainResponseChoices(
                index=0, message=Message(role="assistant",
                                         content="Error from chain server. Please check chain-server logs for more details."),
                finish_reason="[DONE]")])
            yield "data: " + r.model_dump_json() + "\n\n"
        finally:
            METRICS.observe("generate_seconds", time.perf_counter() - t_start)
            tracer.end(span)

    if generator is not None and getattr(generator, "supports_async", False):
        # the request is already queued on the engine (prepare): if the body is never iterated
        # (client gone before the first chunk) the background task still cancels it
        cancel = getattr(generator, "cancel", None)
        return StreamingResponse(response_agen(), media_type="text/event-stream",
                                 background=BackgroundTask(cancel) if cancel else None)
    return StreamingResponse(response_generator(), media_type="text/event-stream")


@app.post("/search", response_model=DocumentSearchResponse)
async def document_search(request: Request, data: DocumentSearch) -> Dict[str, List[Dict[str, Any]]]:
    with tracer.span("POST /search", {"top_k": data.top_k}, _traceparent(request)):
        try:
            example = app.example()
            if hasattr(example, "document_search") and callable(example.document_search):
                result = await asyncio.to_thread(example.document_search, data.query, data.top_k)
                chunks = [DocumentChunk(content=e.get("content", ""), filename=e.get("source", ""),
                                        score=e.get("score", 0.0)) for e in result]
                return DocumentSearchResponse(chunks=chunks)
            raise NotImplementedError("Example class has not implemented the document_search method.")
        except Exception as e:  # noqa: BLE001
            logger.error("Error from POST /search endpoint. Error details: %s", e)
            return JSONResponse(content={"message": "Error occurred while searching documents."}, status_code=500)


@app.get("/documents", response_model=DocumentsResponse)
async def get_documents(request: Request) -> DocumentsResponse:
    try:
        example = app.example()
        if hasattr(example, "get_documents") and callable(example.get_documents):
            return DocumentsResponse(documents=example.get_documents())
        raise NotImplementedError("Example class has not implemented the get_documents method.")
    except Exception as e:  # noqa: BLE001
        logger.error("Error from GET /documents endpoint. Error details: %s", e)
        return JSONResponse(content={"message": "Error occurred while fetching documents."}, status_code=500)


@app.delete("/documents")
async def delete_document(request: Request, filename: str) -> JSONResponse:
    try:
        example = app.example()
        if hasattr(example, "delete_documents") and callable(example.delete_documents):
            if not example.delete_documents([filename]):
                raise Exception(f"Error in deleting document {filename}")
            return JSONResponse(content={"message": f"Document {filename} deleted successfully"}, status_code=200)
        raise NotImplementedError("Example class has not implemented the delete_document method.")
    except Exception as e:  # noqa: BLE001
        logger.error("Error from DELETE /documents endpoint. Error details: %s", e)
        return JSONResponse(content={"message": f"Error deleting document {filename}"}, status_code=500)
