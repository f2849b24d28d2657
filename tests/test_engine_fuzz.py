"""Property-based engine fuzzing (CPU, reference ops): random arrivals with shared prefixes,
beam searches (copy-on-fork KV pages), aborts, tiny KV pools that force preemption, chunked
prefill, mixed prefill+decode steps and pipelined (async) decode — every surviving request
(greedy or beam) must produce exactly the tokens it produces alone, and every KV block must be
back in the pool at the end."""
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine, SamplingParams

BASE = [11, 12, 13, 14, 15, 16, 17, 18] * 9           # 72-token shared prefix (one full page + 8)


@pytest.fixture(scope="module")
def model():
    from nv_genai_amd.models.config import llama_config
    from nv_genai_amd.models.llama import LlamaModel
    from nv_genai_amd.parallel.dist import ParallelContext

    return LlamaModel(llama_config("llama-tiny"), "cpu", pctx=ParallelContext(), seed=9)


_SOLO = {}


def _params(n, beam):
    return SamplingParams(temperature=0.0, max_tokens=n, ignore_eos=True, beam_width=2 if beam else 1)


def _solo(model, prompt, n, beam=False):
    key = (tuple(prompt), n, beam)
    if key not in _SOLO:
        e = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=4, max_batched_tokens=1024, max_model_len=512,
                                   kv_cache_blocks=32, enable_prefix_caching=False), device="cpu", model=model)
        _SOLO[key] = e.generate([prompt], _params(n, beam))[0].output_ids
    return _SOLO[key]


def _near_tie(model, prompt, got, want, tol=0.02):
    """Greedy outputs that differ only because two logits tie to within bf16 rounding: at the
    first differing position, both tokens' logits (recomputed on the shared prefix) are
    within ``tol`` of each other. Batch composition and prefill chunking legitimately change
    the rounding of a random-weight tiny model whose top logits are often 1 ulp apart."""
    from nv_genai_amd.models.llama import AttnMeta

    k = next((i for i, (a, b) in enumerate(zip(got, want)) if a != b), None)
    if k is None:
        return False
    ids = list(prompt) + list(want[:k])
    T = len(ids)
    nb = (T + 63) // 64
    model.allocate_kv_cache(nb, 64)
    meta = AttnMeta(kind="prefill", slots=torch.arange(T, dtype=torch.int32),
                    cu_q=torch.tensor([0, T], dtype=torch.int32), ctx_lens=torch.tensor([T], dtype=torch.int32),
                    block_tables=torch.arange(nb, dtype=torch.int32).unsqueeze(0), max_q_len=T, max_ctx=T)
    with torch.no_grad():
        h = model.forward(torch.tensor(ids, dtype=torch.int32), torch.arange(T, dtype=torch.int32), meta,
                          sample_idx=torch.tensor([T - 1]))
        lg = model.logits(h)[0].float()
    return abs(lg[got[k]].item() - lg[want[k]].item()) <= tol * max(1.0, lg.abs().max().item())


event = st.one_of(
    st.tuples(st.just("add"), st.integers(0, 3), st.integers(1, 60), st.integers(1, 12)),
    st.tuples(st.just("step"), st.integers(1, 4), st.just(0), st.just(0)),
    st.tuples(st.just("abort"), st.integers(0, 20), st.just(0), st.just(0)),
    st.tuples(st.just("beam"), st.integers(0, 3), st.integers(1, 60), st.integers(1, 6)),
)


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(events=st.lists(event, min_size=1, max_size=25), mixed=st.sampled_from([0, 64]),
       async_decode=st.booleans(), mbt=st.sampled_from([40, 128]), blocks=st.sampled_from([10, 24]))
def test_engine_fuzz_matches_solo_and_frees_blocks(model, events, mixed, async_decode, mbt, blocks):
    eng = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=6, max_batched_tokens=mbt, max_model_len=512,
                                 kv_cache_blocks=blocks, mixed_prefill_tokens=mixed, async_decode=async_decode,
                                 token_alignment=1), device="cpu", model=model)
    live, aborted, meta = [], set(), {}
    g = torch.Generator().manual_seed(len(events))
    for kind, a, b, c in events:
        if kind in ("add", "beam"):
            suffix = torch.randint(3, 200, (b,), generator=g).tolist()
            prompt = (BASE[: 8 * (a + 1) + 8 * a] if a else []) + suffix
            r = eng.add_request(prompt, _params(c, kind == "beam"))
            live.append(r)
            meta[r.id] = (prompt, c, kind == "beam")
        elif kind == "step":
            for _ in range(a):
                eng.step()
        elif kind == "abort" and live:
            r = live[a % len(live)]
            if not r.finished:
                eng.abort(r.id)
                aborted.add(r.id)
    eng.run_until_done()
    for r in live:
        if r.id in aborted:
            continue
        prompt, n, beam = meta[r.id]
        want = _solo(model, prompt, n, beam)
        assert r.finished, r.id
        assert r.output_ids == want or (not beam and _near_tie(model, prompt, r.output_ids, want)), \
            (r.id, beam, r.output_ids, want)
    assert eng.sched.used_blocks() == 0, eng.sched.used_blocks()
    assert not eng.has_work()
