"""Distributed tracing (reference: RetrievalAugmentedGeneration/common/tracing.py,
frontend/frontend/tracing.py, tools/observability/*/opentelemetry_callback.py).

OpenTelemetry is not installed here, so this is a small self-contained tracer with the same
observable behaviour:

* enabled by ``ENABLE_TRACING=true``; ``service.name`` per process (chain-server, frontend,
  model-server);
* W3C ``traceparent`` propagation: the frontend injects it into every chain-server call, the
  chain server extracts it so a request's spans share one trace id end to end;
* exporters: OTLP/HTTP JSON to ``OTEL_EXPORTER_OTLP_ENDPOINT`` (``/v1/traces``, batched on a
  background thread), an in-memory exporter (tests), and a console exporter;
* :class:`TracingCallback` — the LangChain/LlamaIndex callback-handler role: spans for chain,
  LLM, retriever, embedding and tool events, first-token latency, token counts, per-token
  events (optional) and psutil process metrics at span end.
"""
from __future__ import annotations

import contextlib
import contextvars
import json
import logging
import os
import queue
import secrets
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Dict, Iterator, List, Optional

log = logging.getLogger(__name__)

_current: contextvars.ContextVar[Optional["Span"]] = contextvars.ContextVar("nga_span", default=None)


def tracing_enabled() -> bool:
    return os.environ.get("ENABLE_TRACING", "false").lower() == "true"


@dataclass
class Span:
    name: str
    trace_id: str
    span_id: str
    parent_id: Optional[str]
    service: str
    start_ns: int = field(default_factory=time.time_ns)
    end_ns: Optional[int] = None
    attributes: Dict[str, Any] = field(default_factory=dict)
    events: List[dict] = field(default_factory=list)
    status: str = "OK"

    def set_attribute(self, k: str, v: Any):
        self.attributes[k] = v

    def add_event(self, name: str, attrs: Optional[dict] = None):
        self.events.append({"name": name, "time_ns": time.time_ns(), "attributes": attrs or {}})

    def record_exception(self, e: BaseException):
        self.status = "ERROR"
        self.add_event("exception", {"exception.type": type(e).__name__, "exception.message": str(e)})

    @property
    def traceparent(self) -> str:
        return f"00-{self.trace_id}-{self.span_id}-01"

    def to_otlp(self) -> dict:
        def kv(d):
            return [{"key": k, "value": {"stringValue": str(v)}} for k, v in d.items()]

        return {"traceId": self.trace_id, "spanId": self.span_id, "parentSpanId": self.parent_id or "",
                "name": self.name, "startTimeUnixNano": str(self.start_ns),
                "endTimeUnixNano": str(self.end_ns or time.time_ns()), "attributes": kv(self.attributes),
                "events": [{"name": e["name"], "timeUnixNano": str(e["time_ns"]), "attributes": kv(e["attributes"])}
                           for e in self.events],
                "status": {"code": 1 if self.status == "OK" else 2}}


class InMemoryExporter:
    def __init__(self):
        self.spans: List[Span] = []

    def export(self, spans: List[Span]):
        self.spans.extend(spans)


class ConsoleExporter:
    def export(self, spans: List[Span]):
        for s in spans:
            log.info("span %s %s %.3fms %s", s.name, s.trace_id, ((s.end_ns or 0) - s.start_ns) / 1e6, s.attributes)


class OTLPHttpExporter:
    """Batched OTLP/HTTP-JSON export on a daemon thread (never blocks the request path)."""

    def __init__(self, endpoint: Optional[str] = None, flush_s: float = 1.0):
        ep = endpoint or os.environ.get("OTEL_EXPORTER_OTLP_ENDPOINT", "http://otel-collector:4318")
        self.url = ep.rstrip("/") + "/v1/traces"
        self.q: "queue.Queue[Span]" = queue.Queue(maxsize=10000)
        self.flush_s = flush_s
        threading.Thread(target=self._run, daemon=True, name="otlp-export").start()

    def export(self, spans: List[Span]):
        for s in spans:
            try:
                self.q.put_nowait(s)
            except queue.Full:
                pass

    def _run(self):
        import requests

        while True:
            batch = [self.q.get()]
            t0 = time.time()
            while time.time() - t0 < self.flush_s and len(batch) < 512:
                try:
                    batch.append(self.q.get(timeout=0.05))
                except queue.Empty:
                    pass
            by_svc: Dict[str, List[Span]] = {}
            for s in batch:
                by_svc.setdefault(s.service, []).append(s)
            body = {"resourceSpans": [
                {"resource": {"attributes": [{"key": "service.name", "value": {"stringValue": svc}}]},
                 "scopeSpans": [{"scope": {"name": "nv_genai_amd"}, "spans": [s.to_otlp() for s in ss]}]}
                for svc, ss in by_svc.items()]}
            try:
                requests.post(self.url, data=json.dumps(body), headers={"Content-Type": "application/json"}, timeout=5)
            except Exception as e:  # noqa: BLE001 - tracing must never break serving
                log.debug("otlp export failed: %s", e)


class Tracer:
    def __init__(self, service: str, exporter=None, enabled: Optional[bool] = None):
        self.service = service
        self.enabled = tracing_enabled() if enabled is None else enabled
        if exporter is None and self.enabled:
            exporter = OTLPHttpExporter() if os.environ.get("OTEL_EXPORTER_OTLP_ENDPOINT") else ConsoleExporter()
        self.exporter = exporter

    def _new(self, name: str, parent: Optional[Span], traceparent: Optional[str]) -> Span:
        trace_id, parent_id = None, None
        if parent is not None:
            trace_id, parent_id = parent.trace_id, parent.span_id
        elif traceparent:
            ctx = parse_traceparent(traceparent)
            if ctx:
                trace_id, parent_id = ctx
        return Span(name, trace_id or secrets.token_hex(16), secrets.token_hex(8), parent_id, self.service)

    @contextlib.contextmanager
    def span(self, name: str, attributes: Optional[dict] = None, traceparent: Optional[str] = None
             ) -> Iterator[Optional[Span]]:
        if not self.enabled:
            yield None
            return
        s = self._new(name, _current.get(), traceparent)
        if attributes:
            s.attributes.update(attributes)
        tok = _current.set(s)
        try:
            yield s
        except BaseException as e:
            s.record_exception(e)
            raise
        finally:
            _current.reset(tok)
            self.end(s)

    def start(self, name: str, parent: Optional[Span] = None, attributes: Optional[dict] = None,
              traceparent: Optional[str] = None) -> Optional[Span]:
        if not self.enabled:
            return None
        s = self._new(name, parent or _current.get(), traceparent)
        if attributes:
            s.attributes.update(attributes)
        return s

    def end(self, s: Optional[Span]):
        if s is None:
            return
        s.end_ns = time.time_ns()
        if self.exporter is not None:
            self.exporter.export([s])


def parse_traceparent(tp: str):
    parts = tp.strip().split("-")
    if len(parts) != 4 or len(parts[1]) != 32 or len(parts[2]) != 16:
        return None
    return parts[1], parts[2]


def inject_context(headers: Optional[dict] = None) -> dict:
    """Carrier for outgoing calls: adds ``traceparent`` of the current span (if any)."""
    headers = dict(headers or {})
    s = _current.get()
    if s is not None:
        headers["traceparent"] = s.traceparent
    return headers


def current_span() -> Optional[Span]:
    return _current.get()


def process_metrics() -> dict:
    try:
        import psutil

        p = psutil.Process()
        with p.oneshot():
            ct = p.cpu_times()
            return {"process.threads": p.num_threads(), "process.rss": p.memory_info().rss,
                    "process.cpu.user": ct.user, "process.cpu.system": ct.system,
                    "process.ctx_switches": sum(p.num_ctx_switches())}
    except Exception:  # noqa: BLE001
        return {}


class TracingCallback:
    """Callback handler for chains (the OpenTelemetryCallbackHandler role): one span per
    chain / llm / retriever / embedding / tool run, parented by run nesting."""

    def __init__(self, tracer: Tracer, token_events: bool = False):
        self.tracer = tracer
        self.token_events = token_events
        self.spans: Dict[str, Span] = {}
        self._first: Dict[str, float] = {}
        self._start: Dict[str, float] = {}
        self._ntok: Dict[str, int] = {}

    def _begin(self, run_id: str, name: str, parent_run_id: Optional[str] = None, **attrs):
        parent = self.spans.get(parent_run_id) if parent_run_id else None
        s = self.tracer.start(name, parent, attrs)
        if s is not None:
            self.spans[run_id] = s
        self._start[run_id] = time.perf_counter()

    def _finish(self, run_id: str, **attrs):
        s = self.spans.pop(run_id, None)
        if s is not None:
            s.attributes.update(attrs)
            s.attributes.update(process_metrics())
            self.tracer.end(s)

    def on_chain_start(self, run_id, name="chain", parent_run_id=None, inputs=None):
        self._begin(run_id, name, parent_run_id, **({"inputs": str(inputs)[:2000]} if inputs else {}))

    def on_chain_end(self, run_id, outputs=None):
        self._finish(run_id, **({"outputs": str(outputs)[:2000]} if outputs is not None else {}))

    def on_llm_start(self, run_id, prompts, parent_run_id=None, **settings):
        self._begin(run_id, "llm", parent_run_id, prompts=str(prompts)[:4000], **settings)
        self._ntok[run_id] = 0

    def on_llm_new_token(self, run_id, token: str):
        if run_id not in self._first:
            self._first[run_id] = time.perf_counter()
        self._ntok[run_id] = self._ntok.get(run_id, 0) + 1
        s = self.spans.get(run_id)
        if s is not None and self.token_events:
            s.add_event("new_token", {"token": token})

    def on_llm_end(self, run_id, output: str = "", prompt_tokens: Optional[int] = None):
        t0 = self._start.pop(run_id, time.perf_counter())
        ft = self._first.pop(run_id, None)
        attrs = {"completion_tokens": self._ntok.pop(run_id, 0), "output": output[:4000]}
        if prompt_tokens is not None:
            attrs["prompt_tokens"] = prompt_tokens
        if ft is not None:
            attrs["first_token_time_ms"] = round(1000 * (ft - t0), 3)
        self._finish(run_id, **attrs)

    def on_llm_error(self, run_id, error: BaseException):
        s = self.spans.get(run_id)
        if s is not None:
            s.record_exception(error)
        self._finish(run_id)

    def on_retriever_start(self, run_id, query: str, parent_run_id=None):
        self._begin(run_id, "retriever", parent_run_id, query=query)

    def on_retriever_end(self, run_id, documents):
        attrs = {}
        for i, d in enumerate(documents or []):
            doc, score = (d if isinstance(d, tuple) else (d, None))
            attrs[f"documents.{i}.content"] = getattr(doc, "page_content", str(doc))[:500]
            if score is not None:
                attrs[f"documents.{i}.score"] = score
        self._finish(run_id, **attrs)

    def on_embedding(self, run_id, batch_size: int, tokens: int = 0, parent_run_id=None):
        self._begin(run_id, "embedding", parent_run_id, batch_size=batch_size, tokens=tokens)
        self._finish(run_id)

    def on_tool_start(self, run_id, tool: str, tool_input: str, parent_run_id=None):
        self._begin(run_id, f"tool:{tool}", parent_run_id, input=tool_input[:2000])

    def on_tool_end(self, run_id, output: str):
        self._finish(run_id, output=str(output)[:2000])

    def on_retry(self, run_id, attempt: int, error: str = ""):
        s = self.spans.get(run_id)
        if s is not None:
            s.add_event("retry", {"attempt": attempt, "error": error})


_TRACERS: Dict[str, Tracer] = {}


def get_tracer(service: str) -> Tracer:
    t = _TRACERS.get(service)
    if t is None:
        t = Tracer(service)
        _TRACERS[service] = t
    return t
