"""Background driver for the LLM engine: one thread steps the continuous-batching engine,
any number of producer threads / asyncio tasks submit requests and consume token streams.

Failure handling (SURVEY.md §5.3 "new framework"): an exception inside a step fails every
in-flight stream with an error instead of hanging it; a watchdog flags a step that runs longer
than ``watchdog_s`` (readiness then reports unhealthy); consumers can cancel (client
disconnect) and the request is aborted in the scheduler, freeing its KV blocks.
"""
from __future__ import annotations

import asyncio
import logging
import os
import queue
import threading
import time
from typing import AsyncIterator, Iterator, List, Optional

from ..engine.llm_engine import LLMEngine, Request, SamplingParams

log = logging.getLogger(__name__)
_END = object()


class EngineError(RuntimeError):
    pass


def _deliver(items):
    for aq, item in items:
        aq.put_nowait(item)


class StreamHandle:
    """Token-delta stream of one request (sync and async iteration).

    The engine thread pushes deltas into a thread-safe queue; an asyncio consumer attaches
    its own asyncio.Queue (fed through ``call_soon_threadsafe``) so no executor thread is
    parked per open stream."""

    def __init__(self, service: "EngineService"):
        self.service = service
        self.q: "queue.Queue" = queue.Queue()
        self.request: Optional[Request] = None
        self.error: Optional[BaseException] = None
        self.done = threading.Event()
        self._lock = threading.Lock()
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self._aq: Optional[asyncio.Queue] = None
        self._buf: List[str] = []       # deltas held back by the stream interval
        self._sent_step = -1            # service step of the last delivery (-1: none yet)
        self._sent_time = 0.0

    def _put(self, item):
        with self._lock:
            if self._aq is not None:
                svc = self.service
                if threading.current_thread() is svc.thread:
                    # engine thread: deliveries of one step go to each event loop in ONE
                    # call_soon_threadsafe (one self-pipe write + one loop wake-up per step,
                    # not one per open stream per token). Text deltas are held for up to
                    # ``stream_interval`` steps (the first one and the end go out at once), so
                    # an open stream costs the event loop one wake-up + one SSE frame per
                    # interval instead of per token.
                    if item is not _END:
                        self._buf.append(item)
                        if self._sent_step >= 0 and svc.steps - self._sent_step < svc.stream_interval:
                            svc._held.add(self)   # flushed by the interval or by time (_flush)
                            return
                    self._release()
                    if item is _END:
                        svc._pending.setdefault(self._loop, []).append((self._aq, _END))
                else:
                    self._loop.call_soon_threadsafe(self._aq.put_nowait, item)
            else:
                self.q.put(item)

    def _release(self):
        """Queue the held deltas for delivery with this step (engine thread, under _lock)."""
        svc = self.service
        if self._buf:
            svc._pending.setdefault(self._loop, []).append((self._aq, "".join(self._buf)))
            self._buf = []
        self._sent_step = svc.steps
        self._sent_time = time.monotonic()
        svc._held.discard(self)

    # engine-thread side
    def _on_token(self, req: Request, delta: str):
        if delta:
            self._put(delta)
        if req.finished and not self.done.is_set():
            if req.finish_reason == "error":   # refused at admission: this stream fails alone
                self.error = EngineError(req.error or "request refused by the engine")
            self.done.set()
            self._put(_END)

    def _fail(self, err: BaseException):
        self.error = err
        if not self.done.is_set():
            self.done.set()
            self._put(_END)

    # consumer side
    def __iter__(self) -> Iterator[str]:
        while True:
            item = self.q.get()
            if item is _END:
                if self.error is not None:
                    raise EngineError(str(self.error))
                return
            yield item

    async def aiter(self, coalesce: bool = False) -> AsyncIterator[str]:
        with self._lock:
            self._loop = asyncio.get_running_loop()
            self._aq = asyncio.Queue()
            while True:
                try:
                    self._aq.put_nowait(self.q.get_nowait())
                except queue.Empty:
                    break
        while True:
            item = await self._aq.get()
            if item is _END:
                if self.error is not None:
                    raise EngineError(str(self.error))
                return
            if coalesce:
                parts, end = [item], False
                while not self._aq.empty():
                    nxt = self._aq.get_nowait()
                    if nxt is _END:
                        end = True
                        break
                    parts.append(nxt)
                yield "".join(parts)
                if end:
                    if self.error is not None:
                        raise EngineError(str(self.error))
                    return
                continue
            yield item

    def text(self) -> str:
        return "".join(self)

    def cancel(self):
        if self.request is not None and not self.done.is_set():
            self.service.abort(self.request.id)
            self._fail(EngineError("cancelled"))

    @property
    def finish_reason(self) -> Optional[str]:
        return None if self.request is None else self.request.finish_reason

    @property
    def usage(self) -> dict:
        r = self.request
        if r is None:
            return {}
        return {"prompt_tokens": len(r.prompt_ids), "completion_tokens": len(r.output_ids),
                "total_tokens": len(r.prompt_ids) + len(r.output_ids)}


class EngineService:
    def __init__(self, engine: LLMEngine, watchdog_s: float = 300.0, name: str = "llm",
                 quiet_gc: bool = True, fail_fast: bool = False, stream_interval: Optional[int] = None,
                 stream_max_hold_ms: Optional[float] = None):
        if quiet_gc:   # no multi-ms GC pauses on the thread that launches GPU steps
            from ..utils.runtime import quiet_gc as _quiet

            _quiet()
        self.engine = engine
        self.watchdog_s = watchdog_s
        # async streams: every token's text goes out with the step that produced it, as the
        # reference streams each chunk as produced (common/server.py:289-301). A throughput
        # deployment may batch deltas over N steps (NGA_STREAM_INTERVAL, opt-in); held text
        # is still flushed within stream_max_hold_s even if its request stalls (preemption)
        self.stream_interval = max(1, int(stream_interval if stream_interval is not None
                                          else os.environ.get("NGA_STREAM_INTERVAL", "1")))
        self.stream_max_hold_s = float(stream_max_hold_ms if stream_max_hold_ms is not None
                                       else os.environ.get("NGA_STREAM_MAX_HOLD_MS", "100")) / 1e3
        self._held: set = set()                      # handles holding deltas back
        self.name = name
        self.cv = threading.Condition()
        self.handles = {}
        self.running = True
        self.step_started: Optional[float] = None
        self.last_error: Optional[str] = None
        self.steps = 0
        self.tasks: "queue.Queue" = queue.Queue()   # callables run on the engine thread
        self._pending: dict = {}                     # event loop -> [(asyncio queue, item)] of this step
        self.fail_fast = fail_fast
        self.thread = threading.Thread(target=self._loop, name=f"{name}-engine", daemon=True)
        self.thread.start()
        if fail_fast:
            threading.Thread(target=self._watchdog, name=f"{name}-watchdog", daemon=True).start()

    def _watchdog(self):
        """Model-parallel replicas: a step stuck past ``watchdog_s`` is a stuck collective (a
        peer rank died or wedged); it cannot be cancelled in-process, so exit and let the
        elastic agent (torchrun --max-restarts) restart the whole TP/PP group with fresh
        RCCL communicators."""
        while self.running:
            time.sleep(min(1.0, self.watchdog_s / 4))
            st = self.step_started
            if st is not None and time.monotonic() - st > self.watchdog_s:
                log.error("engine step stuck for %.0f s: exiting for a group restart", self.watchdog_s)
                logging.shutdown()
                os._exit(70)

    def submit(self, prompt_ids: List[int], params: SamplingParams, mm=None) -> StreamHandle:
        """Queue a request on the engine thread; ``mm``: image features of a vision-language
        prompt (``LLMEngine.add_request``)."""
        h = StreamHandle(self)
        with self.cv:
            req = self.engine.add_request(prompt_ids, params, on_token=h._on_token, mm=mm)
            h.request = req
            self.handles[req.id] = h
            self.cv.notify()
        return h

    def call(self, fn):
        """Run ``fn()`` on the engine thread between two steps and return a Future of its
        result. Model-parallel replicas use this for collectives that must interleave with the
        step broadcasts in the same order on every rank (e.g. a sharded-index search, whose
        command the followers receive through the step channel)."""
        import concurrent.futures as cf

        fut = cf.Future()
        with self.cv:
            self.tasks.put((fn, fut))
            self.cv.notify()
        return fut

    def _run_tasks(self):
        while True:
            try:
                fn, fut = self.tasks.get_nowait()
            except queue.Empty:
                return
            if not fut.set_running_or_notify_cancel():
                continue
            try:
                fut.set_result(fn())
            except BaseException as e:  # noqa: BLE001 - delivered to the caller
                fut.set_exception(e)

    def abort(self, rid: int):
        self.engine.abort(rid)
        self.handles.pop(rid, None)

    def _loop(self):
        while self.running:
            with self.cv:
                while self.running and not self.engine.has_work() and self.tasks.empty():
                    self.cv.wait(timeout=0.5)
            if not self.running:
                break
            if not self.tasks.empty():
                self.engine.drain_and_run(self._run_tasks)
                self._flush()
                if not self.engine.has_work():
                    continue
            try:
                self.step_started = time.monotonic()
                done = self.engine.step()
                self.steps += 1
                for r in done:
                    self.handles.pop(r.id, None)
            except Exception as e:  # noqa: BLE001 - fail the streams, keep serving
                log.exception("engine step failed")
                self.last_error = repr(e)
                for rid, h in list(self.handles.items()):
                    try:
                        self.engine.abort(rid)
                    except Exception:  # noqa: BLE001
                        pass
                    h._fail(e)
                self.handles.clear()
                if self.fail_fast:
                    # model-parallel: the followers' state after a failed step is unknown
                    # (a peer may be dead) -> restart the group rather than limp on
                    log.error("step failed in a model-parallel replica: exiting for a group restart")
                    logging.shutdown()
                    os._exit(70)
            finally:
                self.step_started = None
                self._flush()

    def _flush(self):
        """Hand the step's stream deliveries to their event loops, one callback per loop.
        Deltas held by the stream interval go out once the interval or the hold time has
        passed, whether or not their request produced another token."""
        if self._held:
            now = time.monotonic()
            for h in list(self._held):
                if (self.steps - h._sent_step >= self.stream_interval
                        or now - h._sent_time >= self.stream_max_hold_s):
                    with h._lock:
                        h._release()
        if not self._pending:
            return
        pending, self._pending = self._pending, {}
        for loop, items in pending.items():
            try:
                loop.call_soon_threadsafe(_deliver, items)
            except RuntimeError:   # loop closed (server shutting down): nobody is listening
                pass

    def healthy(self) -> bool:
        st = self.step_started
        return self.thread.is_alive() and not (st is not None and time.monotonic() - st > self.watchdog_s)

    def metrics(self) -> dict:
        e = self.engine
        return {"running": e.sched.num_running(), "waiting": e.sched.num_waiting() + len(e._inbox),
                "kv_usage": e.kv_usage(), "steps": self.steps, **e.stats,
                "prefix_hit_blocks": e.sched.prefix_hits(), "preemptions": e.sched.preemptions()}

    def shutdown(self):
        self.running = False
        with self.cv:
            self.cv.notify_all()
        self.thread.join(timeout=5)
