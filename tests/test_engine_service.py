"""EngineService failure handling (SURVEY.md §5.3 "new framework"), on CPU with the tiny model:
a step that raises fails every in-flight stream with EngineError and the service keeps
serving; a step that overruns the watchdog makes readiness report unhealthy; a cancelled stream
aborts its request and frees its KV blocks."""
import os
import threading
import time

import pytest

from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine, SamplingParams
from nv_genai_amd.serving.engine_service import EngineError, EngineService


@pytest.fixture()
def service():
    eng = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=8, max_batched_tokens=256, max_model_len=512,
                                 kv_cache_blocks=64), device="cpu")
    svc = EngineService(eng, watchdog_s=0.3, quiet_gc=False)
    yield svc
    svc.shutdown()


def _params(n):
    return SamplingParams(temperature=0.0, max_tokens=n, ignore_eos=True)


def test_failed_step_fails_streams_and_service_keeps_serving(service):
    eng = service.engine
    real_step = eng.step
    calls = {"n": 0}

    def flaky_step(*a, **kw):
        calls["n"] += 1
        if calls["n"] == 2:
            raise RuntimeError("injected step failure")
        return real_step(*a, **kw)

    eng.step = flaky_step
    h = service.submit([5, 6, 7, 8] * 4, _params(20))
    with pytest.raises(EngineError, match="injected step failure"):
        h.text()
    assert "injected" in service.last_error
    assert not eng.has_work()                     # the failed request was aborted
    eng.step = real_step
    h2 = service.submit([9, 10, 11], _params(5))
    h2.text()
    assert h2.finish_reason == "length" and len(h2.request.output_ids) == 5
    assert service.healthy()


def test_watchdog_reports_a_stuck_step(service):
    eng = service.engine
    real_step = eng.step
    entered = threading.Event()

    def slow_step(*a, **kw):
        entered.set()
        time.sleep(1.0)
        return real_step(*a, **kw)

    eng.step = slow_step
    h = service.submit([1, 2, 3], _params(1))
    assert entered.wait(5)
    time.sleep(0.5)                               # past watchdog_s = 0.3 inside the step
    assert not service.healthy()
    eng.step = real_step
    h.text()
    deadline = time.time() + 5
    while not service.healthy() and time.time() < deadline:
        time.sleep(0.05)
    assert service.healthy()


def test_cancel_aborts_request_and_frees_blocks(service):
    eng = service.engine
    used0 = eng.sched.used_blocks()
    h = service.submit([3, 4, 5, 6] * 8, _params(400))
    it = iter(h)
    next(it)                                      # the request is running
    h.cancel()
    with pytest.raises(EngineError, match="cancelled"):
        for _ in it:
            pass
    deadline = time.time() + 5
    while eng.has_work() and time.time() < deadline:
        time.sleep(0.02)
    assert h.request.finish_reason == "abort"
    assert not eng.has_work() and eng.sched.used_blocks() == used0
    assert len(h.request.output_ids) < 400


def test_async_streams_batch_deliveries_per_interval():
    """Async consumers get the same text as a sync stream, with text deltas held for up to
    ``stream_interval`` engine steps (first delta and end immediately) and every step's
    deliveries handed to the event loop in one callback."""
    import asyncio

    eng = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=8, max_batched_tokens=256, max_model_len=512,
                                 kv_cache_blocks=64), device="cpu")
    svc = EngineService(eng, quiet_gc=False, stream_interval=4, stream_max_hold_ms=60_000)
    try:
        want = svc.submit([5, 6, 7, 8] * 4, _params(24)).text()

        async def run():
            return await asyncio.gather(*[_collect(h) for h in
                                          [svc.submit([5, 6, 7, 8] * 4, _params(24)) for _ in range(3)]])

        async def _collect(h):
            return [c async for c in h.aiter(coalesce=True)]

        outs = asyncio.run(run())
        for chunks in outs:
            assert "".join(chunks) == want
            assert len(chunks) <= 24 // 4 + 2, chunks
        assert svc._pending == {}
    finally:
        svc.shutdown()


def test_held_deltas_flush_by_time_and_default_is_per_token():
    """The default stream interval is one step (a delta per token, as the reference streams);
    with a long interval, held text still goes out once it has waited stream_max_hold_ms."""
    import asyncio

    eng = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=8, max_batched_tokens=256, max_model_len=512,
                                 kv_cache_blocks=64), device="cpu")
    if "NGA_STREAM_INTERVAL" not in os.environ:
        d = EngineService(eng, quiet_gc=False)
        d.shutdown()
        assert d.stream_interval == 1
    svc = EngineService(eng, quiet_gc=False, stream_interval=1000, stream_max_hold_ms=0)
    try:
        async def run():
            h = svc.submit([5, 6, 7, 8] * 4, _params(12))
            return [c async for c in h.aiter(coalesce=False)]

        chunks = asyncio.run(run())
        assert len(chunks) >= 6, chunks   # not one burst at the end: flushed step by step
    finally:
        svc.shutdown()


def test_add_request_does_not_wait_for_a_running_step():
    """A step holds the engine lock for its whole duration; add_request from another thread
    queues in the inbox instead of blocking, and the next step admits it in arrival order."""
    eng = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=8, max_batched_tokens=256, max_model_len=512,
                                 kv_cache_blocks=64), device="cpu")
    held, release = threading.Event(), threading.Event()

    def hold():
        with eng.lock:
            held.set()
            release.wait(10)

    t = threading.Thread(target=hold)
    t.start()
    held.wait(5)
    t0 = time.perf_counter()
    a = eng.add_request([5, 6, 7], _params(3))
    b = eng.add_request([8, 9, 10], _params(3))
    assert time.perf_counter() - t0 < 0.5
    assert eng.has_work() and a.id not in eng.requests and len(eng._inbox) == 2
    release.set()
    t.join()
    eng.run_until_done([a, b])
    assert len(a.output_ids) == 3 and len(b.output_ids) == 3 and not eng._inbox


def test_inbox_admission_failure_fails_only_that_request(service):
    """A queued request that the scheduler refuses at admission (here: a forced failure of
    sched.add for one id) finishes alone with finish_reason "error" and its stream raises;
    the step goes on and the other streams complete. Empty prompts and duplicate ids are
    refused by add_request itself, before they can wait in the inbox."""
    eng = service.engine
    with pytest.raises(ValueError, match="empty prompt"):
        eng.add_request([], _params(2))
    first = eng.add_request([5, 6, 7], _params(2), request_id=777)
    with pytest.raises(ValueError, match="duplicate"):
        eng.add_request([5, 6, 7], _params(2), request_id=777)
    eng.run_until_done([first])
    real_add = eng.sched.add

    class Sched:   # the native scheduler's add, failing for one id
        def __getattr__(self, k):
            return getattr(real_sched, k)

        def add(self, rid, prompt, max_new):
            if rid == 4242:
                raise RuntimeError("injected admission failure")
            return real_add(rid, prompt, max_new)

    real_sched = eng.sched
    eng.sched = Sched()
    try:
        held, release = threading.Event(), threading.Event()

        def hold():
            with eng.lock:
                held.set()
                release.wait(10)

        t = threading.Thread(target=hold)
        t.start()
        held.wait(5)
        from nv_genai_amd.serving.engine_service import StreamHandle

        ok1 = service.submit([8, 9, 10, 11], _params(4))
        bad = StreamHandle(service)   # a stream on the id the scheduler refuses
        bad2 = eng.add_request([4, 5, 6], _params(4), request_id=4242, on_token=bad._on_token)
        bad.request = bad2
        ok2 = service.submit([12, 13, 14], _params(4))
        release.set()
        t.join()
        assert len(ok1.text()) >= 0 and len(ok2.text()) >= 0
        with pytest.raises(EngineError, match="injected admission failure"):
            bad.text()
        assert bad2.finished and bad2.finish_reason == "error"
        assert ok1.request.finished and ok1.request.finish_reason == "length"
        assert ok2.request.finished and ok2.request.finish_reason == "length"
    finally:
        eng.sched = real_sched


def test_prepared_stream_never_consumed_is_cancelled(service):
    """The chain server queues a request on the engine before its response body starts
    (LLMStream.prepare); a client that disconnects before the first chunk never iterates the
    body, so the response's background task cancels the prepared request instead of letting
    it decode to max_tokens with nobody reading (chain_server/server.py generate_answer)."""
    from nv_genai_amd.connectors.local import LocalChatModel
    from nv_genai_amd.examples.common import LLMStream
    from nv_genai_amd.observability.tracing import TracingCallback, get_tracer

    llm = LocalChatModel(service, "local", max_tokens=400, temperature=0.1)
    s = LLMStream(TracingCallback(get_tracer("test")), llm, [{"role": "user", "content": "hello there"}], {})
    s.prepare()
    h = s._handle
    assert h is not None and not h.done.is_set()
    s.cancel()
    assert h.done.is_set() and h.request.finish_reason == "abort"
    deadline = time.time() + 5
    while service.engine.sched.num_running() + service.engine.sched.num_waiting() and time.time() < deadline:
        time.sleep(0.02)
    assert service.engine.sched.num_running() == 0 and service.engine.sched.num_waiting() == 0
    s.cancel()   # idempotent once done


def test_stack_sampler_separates_busy_and_parked_threads(tmp_path):
    """The serving processes' stack sampler (NGA_PY_SAMPLE_OUT): a spinning thread reads as
    busy with its hot function on top, a thread parked on an Event as idle, and the JSON
    summary lands on disk."""
    import json
    import threading
    import time

    from nv_genai_amd.observability.sampler import StackSampler

    stop = threading.Event()

    def spin_here():
        x = 0
        while not stop.is_set():
            x += 1

    busy = threading.Thread(target=spin_here, name="spinner", daemon=True)
    parked = threading.Thread(target=stop.wait, name="parked", daemon=True)
    busy.start()
    parked.start()
    s = StackSampler(str(tmp_path / "s.json"), interval_s=0.002).start()
    t_end = time.monotonic() + 5.0     # the spinner competes for the GIL: wait for enough samples
    while s.samples < 30 and time.monotonic() < t_end:
        time.sleep(0.05)
    stop.set()
    s.stop()
    d = json.load(open(tmp_path / "s.json"))
    th = d["threads"]
    assert d["samples"] >= 20
    assert th["spinner"]["busy_share"] > 0.5
    assert any("spin_here" in where for where, _ in th["spinner"]["top_leaf"])
    assert th["parked"]["busy_share"] < 0.2
