"""EngineService failure handling (SURVEY.md §5.3 "new framework"), on CPU with the tiny model:
a step that raises fails every in-flight stream with EngineError and the service keeps
serving; a step that overruns the watchdog makes readiness report unhealthy; a cancelled stream
aborts its request and frees its KV blocks."""
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
    svc = EngineService(eng, quiet_gc=False, stream_interval=4)
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
