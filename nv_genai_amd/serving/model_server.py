"""OpenAI / NIM-compatible model server (SURVEY.md §7.1 ``model_server``): the endpoints the
reference's connectors (ChatNVIDIA, NVIDIAEmbeddings, NeMo Retriever reranking) call, served
by this framework's engines on MI355X.

* ``POST /v1/chat/completions`` — Llama-3 chat template, SSE streaming (``chat.completion.chunk``
  frames then ``data: [DONE]``) or one JSON response; temperature / top_p / top_k / max_tokens /
  stop / seed / repetition_penalty / ignore_eos / logprobs;
* ``POST /v1/completions`` — raw prompt completion (same knobs);
* ``POST /v1/embeddings`` — ``input`` str|list, ``input_type`` query|passage, ``truncate``
  END|START|NONE, float or base64 encoding; requests are merged by a dynamic batcher;
* ``POST /v1/ranking`` — ``{query:{text}, passages:[{text}]}`` -> ``rankings[{index, logit}]``;
* ``GET /v1/models``, ``GET /v1/health/ready``, ``GET /v1/health/live``, ``GET /metrics``.

``python -m nv_genai_amd.serving.model_server --llm llama3-8b --embed arctic-embed-l --port 8000``
"""
from __future__ import annotations

import argparse
import asyncio
import dataclasses
import base64
import json
import logging
import os
import time
import uuid
from typing import Any, Dict, List, Optional, Union

import torch

from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, PlainTextResponse, StreamingResponse
from pydantic import BaseModel, Field

from ..engine.llm_engine import SamplingParams
from ..observability.metrics import Registry
from ..observability.tracing import get_tracer

log = logging.getLogger(__name__)


class ChatMessage(BaseModel):
    role: str = "user"
    content: Union[str, List[Dict[str, Any]]] = ""


class ChatRequest(BaseModel):
    model: str = ""
    messages: List[ChatMessage]
    temperature: float = Field(0.2, ge=0.0, le=2.0)
    top_p: float = Field(0.7, gt=0.0, le=1.0)
    top_k: int = Field(0, ge=0)
    max_tokens: int = Field(1024, ge=1)
    stop: Optional[Union[str, List[str]]] = None
    seed: Optional[int] = None
    stream: bool = False
    repetition_penalty: float = Field(1.0, gt=0.0)
    ignore_eos: bool = False
    logprobs: bool = False
    frequency_penalty: float = Field(0.0, ge=-2.0, le=2.0)
    presence_penalty: float = Field(0.0, ge=-2.0, le=2.0)
    beam_width: int = Field(1, ge=1, le=16)
    length_penalty: float = 1.0
    response_format: Optional[Dict[str, Any]] = None   # {"type": "json_object"} constrains to JSON
    n: int = Field(1, ge=1, le=16)   # choices per prompt (parallel sampling, or the top-n beams)


class CompletionRequest(BaseModel):
    model: str = ""
    prompt: Union[str, List[str]]
    temperature: float = Field(0.2, ge=0.0, le=2.0)
    top_p: float = Field(0.7, gt=0.0, le=1.0)
    top_k: int = Field(0, ge=0)
    max_tokens: int = Field(16, ge=1)
    stop: Optional[Union[str, List[str]]] = None
    seed: Optional[int] = None
    stream: bool = False
    repetition_penalty: float = Field(1.0, gt=0.0)
    ignore_eos: bool = False
    frequency_penalty: float = Field(0.0, ge=-2.0, le=2.0)
    presence_penalty: float = Field(0.0, ge=-2.0, le=2.0)
    beam_width: int = Field(1, ge=1, le=16)
    length_penalty: float = 1.0
    response_format: Optional[Dict[str, Any]] = None   # {"type": "json_object"} constrains to JSON
    n: int = Field(1, ge=1, le=16)   # choices per prompt (parallel sampling, or the top-n beams)


class EmbeddingRequest(BaseModel):
    input: Union[str, List[str]]
    model: str = ""
    input_type: str = "passage"
    truncate: str = "END"
    encoding_format: str = "float"


class RankText(BaseModel):
    text: str


class RankingRequest(BaseModel):
    model: str = ""
    query: RankText
    passages: List[RankText]
    truncate: str = "END"


def _params(r) -> SamplingParams:
    stop = [r.stop] if isinstance(r.stop, str) else list(r.stop or [])
    return SamplingParams(temperature=r.temperature, top_p=r.top_p, top_k=r.top_k, max_tokens=r.max_tokens,
                          stop=stop, seed=r.seed, repetition_penalty=r.repetition_penalty,
                          ignore_eos=r.ignore_eos, logprobs=getattr(r, "logprobs", False),
                          frequency_penalty=r.frequency_penalty, presence_penalty=r.presence_penalty,
                          beam_width=r.beam_width, length_penalty=r.length_penalty,
                          response_format=(r.response_format or {}).get("type"))


def _content_text(c) -> str:
    if isinstance(c, str):
        return c
    return "".join(p.get("text", "") for p in c if isinstance(p, dict) and p.get("type", "text") == "text")


def _has_images(messages) -> bool:
    return any(isinstance(m.content, list) and any(isinstance(p, dict) and p.get("type") in ("image_url", "image")
                                                   for p in m.content) for m in messages)


def create_app(llm_service=None, embed_engine=None, rerank_engine=None, llm_name: str = "meta/llama3-8b-instruct",
               embed_name: str = "snowflake/arctic-embed-l", rerank_name: str = "nv-rerank-qa-mistral-4b:1",
               batch_delay_s: float = 0.002, vlm=None, vlm_service=None, vlm_name: str = "ai-neva-22b",
               deplot=None, deplot_names=("google/deplot", "ai-google-deplot"), reward=None,
               reward_name: str = "nvidia/nemotron-4-340b-reward", max_inflight: Optional[int] = None) -> FastAPI:
    """``vlm`` / ``vlm_service``: a :class:`~nv_genai_amd.models.vision.VisionLanguageModel`
    and the :class:`EngineService` over its engine; chat requests with ``image_url`` parts
    (or ``model == vlm_name``) go there — the NeVA / DePlot endpoint contract of the
    reference's multimodal example (examples/multimodal_rag/llm/llm_client.py:37-42).
    ``deplot``: a :class:`~nv_genai_amd.models.pix2struct.DePlot` chart-to-table model; chat
    requests naming one of ``deplot_names`` are answered by it (the images of the request, its
    text as the rendered header prompt; custom_pdf_parser.py:55-71). ``reward``: a
    :class:`~nv_genai_amd.models.reward.RewardModel`; chat requests naming ``reward_name``
    score their last user / assistant turns and answer "helpfulness:x,correctness:y,..." (the
    reward endpoint the KG-RAG evaluation calls, evaluation.py:38-56). ``max_inflight`` (default
    ``NGA_MAX_INFLIGHT``, 0 = no limit): load shedding — a generation request that would take the
    LLM service past this many in-flight sequences gets 429 with ``Retry-After`` instead of
    queueing without bound behind the running batch."""
    app = FastAPI(title="nv_genai_amd model server")
    if max_inflight is None:
        max_inflight = int(os.environ.get("NGA_MAX_INFLIGHT", "0"))
    app.state.max_inflight = max_inflight
    metrics = Registry()

    from .engine_service import EngineError

    @app.exception_handler(EngineError)
    async def _engine_error(request: Request, exc: EngineError):
        # a failed engine step (non-streaming request): 503 + the OpenAI error object
        metrics.inc("engine_errors_total")
        return JSONResponse({"error": {"message": str(exc), "type": "engine_error"}}, status_code=503)
    tracer = get_tracer("model-server")
    batcher = None
    if embed_engine is not None:
        from .batcher import DynamicBatcher

        batcher = DynamicBatcher(embed_engine, batch_delay_s)
    app.state.llm, app.state.embed, app.state.rerank, app.state.batcher = llm_service, embed_engine, rerank_engine, batcher
    app.state.vlm, app.state.vlm_service = vlm, vlm_service
    app.state.deplot = deplot
    app.state.reward = reward
    deplot_batcher = None
    if deplot is not None:
        from ..models.pix2struct import DePlotBatcher

        # concurrent chart requests share one encoder pass and one batched graph decode
        deplot_batcher = DePlotBatcher(deplot)
    app.state.deplot_batcher = deplot_batcher

    def _deplot_run(msgs, max_tokens):
        from ..models.vision import split_image_parts

        texts, images = [], []
        for m in msgs:
            parts, imgs = split_image_parts(m.content)
            texts += [p for p in parts if isinstance(p, str) and p.strip()]
            images += imgs
        if not images:
            raise ValueError("a DePlot request needs at least one image")
        futs = [deplot_batcher.submit(im, " ".join(texts) or None, min(max_tokens, 512)) for im in images]
        return "\n".join(f.result() for f in futs)

    def _shed(svc, n: int = 1):
        """429 response when admitting ``n`` more sequences would exceed ``max_inflight``."""
        cap = app.state.max_inflight
        if cap and len(svc.handles) + n > cap:
            metrics.inc("shed_requests_total")
            return JSONResponse({"error": {"message": f"server busy: {len(svc.handles)} sequences in flight "
                                                      f"(limit {cap})", "type": "rate_limit_exceeded"}},
                                status_code=429, headers={"Retry-After": "1"})
        return None

    def _need(x, what):
        if x is None:
            raise RuntimeError(f"no {what} model loaded on this server")
        return x

    async def _run_stream(handle, rid: str, model: str, obj: str, chat: bool, t0: float):
        first = True
        created = int(time.time())
        # every token frame is the same JSON around its text: built once per stream, the delta
        # spliced in (byte-identical to json.dumps of the chunk, without a dict + encode per token)
        mark = "\x00"
        ch = ({"index": 0, "delta": {"role": "assistant", "content": mark}, "finish_reason": None} if chat
              else {"index": 0, "text": mark, "finish_reason": None})
        head, tail = ("data: " + json.dumps({"id": rid, "object": obj, "created": created, "model": model,
                                             "choices": [ch]}) + "\n\n").split(json.dumps(mark))
        try:
            async for delta in handle.aiter():
                if first:
                    metrics.observe("ttft_seconds", time.perf_counter() - t0)
                    first = False
                yield head + json.dumps(delta) + tail
            fin = {"index": 0, "finish_reason": handle.finish_reason or "stop"}
            fin.update({"delta": {}} if chat else {"text": ""})
            yield "data: " + json.dumps({"id": rid, "object": obj, "created": created, "model": model,
                                         "choices": [fin], "usage": handle.usage}) + "\n\n"
            yield "data: [DONE]\n\n"
        except asyncio.CancelledError:  # client went away: free the sequence
            handle.cancel()
            raise
        except Exception as e:  # noqa: BLE001
            yield "data: " + json.dumps({"error": {"message": str(e), "type": "engine_error"}}) + "\n\n"
        finally:
            metrics.observe("request_seconds", time.perf_counter() - t0)
            r = handle.request
            if r is not None and r.output_ids and r.first_token_time and r.finish_time and len(r.output_ids) > 1:
                metrics.observe("tpot_seconds", (r.finish_time - r.first_token_time) / (len(r.output_ids) - 1))

    async def _complete(handle, t0: float) -> str:
        out = []
        async for d in handle.aiter():
            out.append(d)
        metrics.observe("request_seconds", time.perf_counter() - t0)
        return "".join(out)

    def _submit_n(svc, ids, req):
        """``n`` choices: one beam-search request returns its top-n beams; otherwise n
        sampled sequences over the shared prompt (prefix-cached KV), seeds seed + i."""
        params = _params(req)
        if req.n == 1 or params.beam_width > 1:
            return [svc.submit(ids, params)]
        out = []
        for i in range(req.n):
            seed = None if params.seed is None else params.seed + i
            out.append(svc.submit(ids, dataclasses.replace(params, seed=seed)))
        return out

    def _usage(handles):
        u = {"prompt_tokens": sum(h.usage.get("prompt_tokens", 0) for h in handles),
             "completion_tokens": sum(h.usage.get("completion_tokens", 0) for h in handles)}
        u["total_tokens"] = u["prompt_tokens"] + u["completion_tokens"]
        return u

    def _texts(handle, text, n):
        """The choice texts of one request: its beams (beam search) or its one output."""
        r = handle.request
        if r is not None and r.beams and n > 1:
            return [b[2] for b in r.beams[:n]]
        return [text]

    @app.post("/v1/chat/completions")
    async def chat(req: ChatRequest, request: Request):
        t0 = time.perf_counter()
        metrics.inc("chat_requests_total")
        if req.stream and req.n > 1:
            return JSONResponse({"error": "stream supports n = 1"}, status_code=400)
        if app.state.reward is not None and req.model == reward_name:
            from ..models.reward import format_scores

            q = next((_content_text(m.content) for m in reversed(req.messages) if m.role == "user"), "")
            a = next((_content_text(m.content) for m in reversed(req.messages) if m.role == "assistant"), "")
            with tracer.span("chat.completions.reward", {"model": req.model}, request.headers.get("traceparent")):
                sc = await asyncio.get_running_loop().run_in_executor(None, app.state.reward.score, q, a)
            metrics.observe("request_seconds", time.perf_counter() - t0)
            return {"id": f"chatcmpl-{uuid.uuid4().hex}", "object": "chat.completion", "created": int(time.time()),
                    "model": req.model, "choices": [{"index": 0, "message": {"role": "assistant",
                                                                             "content": format_scores(sc)},
                                                     "finish_reason": "stop"}],
                    "usage": {"prompt_tokens": 0, "completion_tokens": 0, "total_tokens": 0}}
        if app.state.deplot is not None and req.model in deplot_names:
            with tracer.span("chat.completions.deplot", {"model": req.model}, request.headers.get("traceparent")):
                try:
                    text = await asyncio.get_running_loop().run_in_executor(None, _deplot_run, req.messages,
                                                                            req.max_tokens)
                except ValueError as e:
                    return JSONResponse({"error": str(e)}, status_code=400)
            metrics.observe("request_seconds", time.perf_counter() - t0)
            rid = f"chatcmpl-{uuid.uuid4().hex}"
            if req.stream:
                def one():
                    for ch in ({"index": 0, "delta": {"role": "assistant", "content": text}, "finish_reason": None},
                               {"index": 0, "delta": {}, "finish_reason": "stop"}):
                        yield "data: " + json.dumps({"id": rid, "object": "chat.completion.chunk",
                                                     "created": int(time.time()), "model": req.model,
                                                     "choices": [ch]}) + "\n\n"
                    yield "data: [DONE]\n\n"

                return StreamingResponse(one(), media_type="text/event-stream")
            return {"id": rid, "object": "chat.completion", "created": int(time.time()), "model": req.model,
                    "choices": [{"index": 0, "message": {"role": "assistant", "content": text},
                                 "finish_reason": "stop"}],
                    "usage": {"prompt_tokens": 0, "completion_tokens": 0, "total_tokens": 0}}
        use_vlm = app.state.vlm is not None and (_has_images(req.messages) or req.model == vlm_name)
        if use_vlm:
            svc = app.state.vlm_service
            with tracer.span("chat.completions.vision", {"model": req.model}, request.headers.get("traceparent")):
                msgs = [{"role": m.role, "content": m.content} for m in req.messages]
                ids, mm = await asyncio.get_running_loop().run_in_executor(None, app.state.vlm.build_request, msgs)
                handles = [svc.submit(ids, _params(req), mm=mm)]
        else:
            if _has_images(req.messages):
                return JSONResponse({"error": "this server hosts no vision-language model"}, status_code=400)
            svc = _need(app.state.llm, "LLM")
            busy = _shed(svc, req.n)
            if busy is not None:
                return busy
            msgs = [{"role": m.role, "content": _content_text(m.content)} for m in req.messages]
            with tracer.span("chat.completions", {"model": req.model}, request.headers.get("traceparent")):
                # off the event loop: a RAG prompt is ~1,200 tokens of encoding (GIL-free)
                ids = await asyncio.to_thread(svc.engine.apply_chat_template, msgs)
                handles = _submit_n(svc, ids, req)
        rid = f"chatcmpl-{uuid.uuid4().hex}"
        model = req.model or llm_name
        if req.stream:
            return StreamingResponse(_run_stream(handles[0], rid, model, "chat.completion.chunk", True, t0),
                                     media_type="text/event-stream")
        choices = []
        for h in handles:
            text = await _complete(h, t0)
            for t in _texts(h, text, req.n):
                choice = {"index": len(choices), "message": {"role": "assistant", "content": t},
                          "finish_reason": h.finish_reason}
                if req.logprobs and h.request is not None:
                    choice["logprobs"] = {"content": [{"logprob": lp} for lp in h.request.logprobs]}
                choices.append(choice)
        return {"id": rid, "object": "chat.completion", "created": int(time.time()), "model": model,
                "choices": choices, "usage": _usage(handles)}

    @app.post("/v1/completions")
    async def completions(req: CompletionRequest, request: Request):
        svc = _need(app.state.llm, "LLM")
        t0 = time.perf_counter()
        metrics.inc("completion_requests_total")
        prompts = [req.prompt] if isinstance(req.prompt, str) else req.prompt
        tok = svc.engine.tok
        model = req.model or llm_name
        rid = f"cmpl-{uuid.uuid4().hex}"
        if req.stream and (len(prompts) != 1 or req.n > 1):
            return JSONResponse({"error": "stream supports a single prompt and n = 1"}, status_code=400)
        busy = _shed(svc, len(prompts) * req.n)
        if busy is not None:
            return busy
        handles = [h for p in prompts for h in _submit_n(svc, [tok.bos_id] + tok.encode(p), req)]
        if req.stream:
            return StreamingResponse(_run_stream(handles[0], rid, model, "text_completion", False, t0),
                                     media_type="text/event-stream")
        choices = []
        for h in handles:
            text = await _complete(h, t0)
            for t in _texts(h, text, req.n):
                choices.append({"index": len(choices), "text": t, "finish_reason": h.finish_reason})
        return {"id": rid, "object": "text_completion", "created": int(time.time()), "model": model,
                "choices": choices, "usage": _usage(handles)}

    @app.post("/v1/embeddings")
    async def embeddings(req: EmbeddingRequest):
        eng = _need(app.state.embed, "embedding")
        t0 = time.perf_counter()
        texts = [req.input] if isinstance(req.input, str) else list(req.input)
        if req.input_type not in ("query", "passage"):
            return JSONResponse({"error": "input_type must be 'query' or 'passage'"}, status_code=400)
        try:
            seqs = eng.tokenize(texts, req.input_type, req.truncate)
        except ValueError as e:
            return JSONResponse({"error": str(e)}, status_code=400)
        fut = app.state.batcher.submit_ids(seqs)
        vecs = await asyncio.wrap_future(fut)   # host tensors: the batcher waited on its own stream
        metrics.observe("embed_seconds", time.perf_counter() - t0)
        metrics.inc("embed_texts_total", len(texts))
        data = []
        for i, v in enumerate(vecs):
            if req.encoding_format == "base64":   # little-endian fp32, as the OpenAI API encodes it
                emb: Any = base64.b64encode(v.float().numpy().astype("<f4").tobytes()).decode()
            else:
                emb = v.tolist()
            data.append({"object": "embedding", "index": i, "embedding": emb})
        ntok = sum(len(s) for s in seqs)
        return {"object": "list", "data": data, "model": req.model or embed_name,
                "usage": {"prompt_tokens": ntok, "total_tokens": ntok}}

    @app.post("/v1/ranking")
    async def ranking(req: RankingRequest):
        eng = app.state.rerank or _need(app.state.embed, "reranking")
        t0 = time.perf_counter()
        logits = await asyncio.to_thread(eng.rerank, req.query.text, [p.text for p in req.passages], req.truncate)
        metrics.observe("rank_seconds", time.perf_counter() - t0)
        order = sorted(range(len(logits)), key=lambda i: -logits[i])
        return {"rankings": [{"index": i, "logit": float(logits[i])} for i in order]}

    # Triton "generate" extension (the TRT-LLM ensemble contract of
    # experimental/AzureML/trt_llm_azureml.py:282-320): text_input + sampling knobs.
    def _triton_params(b: dict) -> SamplingParams:
        if not 1 <= int(b.get("beam_width", 1)) <= 16:
            raise ValueError("beam_width must be in [1, 16]")
        stop = b.get("stop_words") or []
        return SamplingParams(temperature=float(b.get("temperature", 1.0)), top_p=float(b.get("top_p", 1.0)),
                              top_k=int(b.get("top_k", 0)), max_tokens=int(b.get("max_tokens", 64)),
                              repetition_penalty=float(b.get("repetition_penalty", 1.0)),
                              seed=b.get("random_seed"), stop=[stop] if isinstance(stop, str) else list(stop),
                              ignore_eos=bool(b.get("ignore_eos", False)),
                              beam_width=int(b.get("beam_width", 1)),
                              length_penalty=float(b.get("length_penalty", 1.0)))

    @app.post("/v2/models/{model}/generate")
    async def triton_generate(model: str, request: Request):
        svc = _need(app.state.llm, "LLM")
        b = await request.json()
        try:
            params = _triton_params(b)
        except ValueError as e:
            return JSONResponse({"error": str(e)}, status_code=400)
        tok = svc.engine.tok
        h = svc.submit([tok.bos_id] + tok.encode(b.get("text_input", "")), params)
        text = await _complete(h, time.perf_counter())
        return {"model_name": model, "model_version": "1", "text_output": text}

    @app.post("/v2/models/{model}/generate_stream")
    async def triton_generate_stream(model: str, request: Request):
        svc = _need(app.state.llm, "LLM")
        b = await request.json()
        try:
            params = _triton_params(b)
        except ValueError as e:
            return JSONResponse({"error": str(e)}, status_code=400)
        tok = svc.engine.tok
        h = svc.submit([tok.bos_id] + tok.encode(b.get("text_input", "")), params)

        async def gen():
            async for d in h.aiter():
                yield "data: " + json.dumps({"model_name": model, "model_version": "1", "text_output": d}) + "\n\n"

        return StreamingResponse(gen(), media_type="text/event-stream")

    @app.get("/v1/models")
    def models():
        out = []
        if app.state.llm is not None:
            out.append({"id": llm_name, "object": "model", "owned_by": "nv_genai_amd"})
        if app.state.vlm is not None:
            out.append({"id": vlm_name, "object": "model", "owned_by": "nv_genai_amd"})
        if app.state.deplot is not None:
            out.append({"id": deplot_names[0], "object": "model", "owned_by": "nv_genai_amd"})
        if app.state.embed is not None:
            out.append({"id": embed_name, "object": "model", "owned_by": "nv_genai_amd"})
        if app.state.rerank is not None:
            out.append({"id": rerank_name, "object": "model", "owned_by": "nv_genai_amd"})
        if app.state.reward is not None:
            out.append({"id": reward_name, "object": "model", "owned_by": "nv_genai_amd"})
        return {"object": "list", "data": out}

    @app.get("/v1/health/live")
    def live():
        return {"object": "health-response", "message": "Service is live."}

    @app.get("/v1/health/ready")
    def ready():
        ok = app.state.llm is None or app.state.llm.healthy()
        return JSONResponse({"object": "health-response", "message": "Service is ready." if ok else "not ready"},
                            status_code=200 if ok else 503)

    @app.get("/v1/debug/timeline")
    def timeline(last: int = 256):
        """Recent engine steps (kind, rows, tokens, decode rows, queue depths)."""
        svc = _need(app.state.llm, "LLM")
        return {"steps": svc.engine.timeline(last)}

    @app.get("/metrics")
    def prom():
        g = app.state.llm.metrics() if app.state.llm is not None else {}
        if app.state.batcher is not None:
            g["embed_batches"] = app.state.batcher.batches
        return PlainTextResponse(metrics.render(g, prefix="model_server"), media_type="text/plain; version=0.0.4")

    return app


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--llm", default="llama3-8b", help="LLM preset ('' to disable)")
    ap.add_argument("--embed", default="arctic-embed-l", help="encoder preset ('' to disable)")
    ap.add_argument("--rerank", default="", help="reranker preset ('' to disable)")
    ap.add_argument("--vlm", default="", help="vision-language preset, e.g. neva-22b ('' to disable)")
    ap.add_argument("--deplot", default="", help="Pix2Struct chart-to-table preset, e.g. deplot ('' to disable)")
    ap.add_argument("--reward", default="", help="reward model served as nvidia/nemotron-4-340b-reward, e.g. "
                    "nvidia/nemotron-4-340b-reward or reward-small ('' to disable)")
    ap.add_argument("--weights", default="", help="safetensors dir for the LLM")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--max-num-seqs", type=int, default=256)
    ap.add_argument("--max-inflight", type=int, default=None,
                    help="429 beyond this many in-flight sequences (default NGA_MAX_INFLIGHT, 0 = no limit)")
    ap.add_argument("--max-model-len", type=int, default=8192)
    ap.add_argument("--kv-cache-fraction", type=float, default=0.3)
    ap.add_argument("--kv-cache-dtype", default="auto", choices=("auto", "fp8"),
                    help="fp8: e4m3fn KV pages (twice the cached tokens)")
    ap.add_argument("--fp8", action="store_true", help="W8A8 FP8 projections")
    ap.add_argument("--device", default=None)
    args = ap.parse_args(argv)
    import uvicorn

    from ..observability.sampler import start_from_env

    start_from_env("model")   # NGA_PY_SAMPLE_OUT: stack-sample this process (diagnostics)

    from ..engine.embed_engine import EmbeddingEngine
    from ..engine.llm_engine import EngineConfig, LLMEngine
    from .engine_service import EngineService

    svc = emb = rr = None
    if args.llm:
        weights = None
        if args.weights:
            from ..utils.checkpoint import load_weights

            weights = load_weights(args.weights)
        eng = LLMEngine(EngineConfig(model=args.llm, max_num_seqs=args.max_num_seqs, max_model_len=args.max_model_len,
                                     kv_cache_fraction=args.kv_cache_fraction,
                                     kv_cache_dtype=args.kv_cache_dtype, fp8=args.fp8),
                        device=args.device, weights=weights)
        svc = EngineService(eng)
    if args.embed:
        emb = EmbeddingEngine(args.embed, device=args.device)
    if args.rerank:
        rr = EmbeddingEngine(args.rerank, device=args.device)
    vlm = vsvc = None
    if args.vlm:
        from ..models.vision import VisionLanguageModel, vlm_config

        vc = vlm_config(args.vlm)
        vlm = VisionLanguageModel(vc, device=args.device, engine_cfg=EngineConfig(
            model=vc.llm, max_num_seqs=args.max_num_seqs, max_model_len=args.max_model_len,
            kv_cache_fraction=args.kv_cache_fraction))
        vsvc = EngineService(vlm.engine, name="vlm")
    dp = None
    if args.deplot:
        from ..models.pix2struct import DePlot

        dp = DePlot(args.deplot, device=args.device)
    rw = None
    if args.reward:
        from ..models.reward import RewardModel

        rw = RewardModel(args.reward, device=args.device or ("cuda" if torch.cuda.is_available() else "cpu"))
    app = create_app(svc, emb, rr, vlm=vlm, vlm_service=vsvc, vlm_name=f"ai-{args.vlm}" if args.vlm else "ai-neva-22b",
                     deplot=dp, reward=rw, max_inflight=args.max_inflight)
    uvicorn.run(app, host=args.host, port=args.port, log_level=os.environ.get("LOGLEVEL", "info").lower())


if __name__ == "__main__":
    main()
