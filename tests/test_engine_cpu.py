"""LLM / embedding engine behaviour on CPU (reference ops): continuous batching equals
sequential greedy decoding, stop handling, chunked prefill, prefix caching, sampling."""
import pytest
import torch

from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine, SamplingParams
from nv_genai_amd.ops import reference as ref


@pytest.fixture(scope="module")
def model():
    from nv_genai_amd.models.config import llama_config
    from nv_genai_amd.models.llama import LlamaModel
    from nv_genai_amd.parallel.dist import ParallelContext

    return LlamaModel(llama_config("llama-tiny"), "cpu", pctx=ParallelContext(), seed=3)


def _engine(model, **kw):
    cfg = dict(model="llama-tiny", max_num_seqs=8, max_batched_tokens=96, max_model_len=512, kv_cache_blocks=64)
    cfg.update(kw)
    return LLMEngine(EngineConfig(**cfg), device="cpu", model=model)


PROMPTS = [[3, 4, 5, 6] * 25, [7, 8] * 40, [9] * 5]


def test_batched_equals_sequential(model):
    p = SamplingParams(temperature=0.0, max_tokens=10, ignore_eos=True)
    batched = [r.output_ids for r in _engine(model).generate(PROMPTS, p)]
    for prompt, out in zip(PROMPTS, batched):
        solo = _engine(model, max_batched_tokens=512).generate([prompt], p)[0].output_ids
        assert solo == out


def test_chunked_prefill_matches_unchunked(model):
    p = SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True)
    a = _engine(model, max_batched_tokens=32).generate([PROMPTS[0]], p)[0].output_ids
    b = _engine(model, max_batched_tokens=512).generate([PROMPTS[0]], p)[0].output_ids
    assert a == b


def test_prefix_cache_reuse_is_exact(model):
    e = _engine(model)
    p = SamplingParams(temperature=0.0, max_tokens=5, ignore_eos=True)
    first = e.generate([PROMPTS[0]], p)[0]
    second = e.generate([PROMPTS[0]], p)[0]
    assert second.cached_prefix >= 64 and first.output_ids == second.output_ids


def test_seeded_sampling_reproducible(model):
    p = SamplingParams(temperature=0.9, top_p=0.95, top_k=50, max_tokens=8, ignore_eos=True, seed=1234)
    a = _engine(model).generate([PROMPTS[1]], p)[0].output_ids
    b = _engine(model).generate([PROMPTS[1]], p)[0].output_ids
    assert a == b


def test_stop_token_and_length(model):
    e = _engine(model)
    p = SamplingParams(temperature=0.0, max_tokens=10, ignore_eos=True)
    out = e.generate([PROMPTS[2]], p)[0]
    # stop on the first token that did not already occur earlier in the greedy output
    k = next(i for i in range(1, 10) if out.output_ids[i] not in out.output_ids[:i])
    tok = out.output_ids[k]
    r = e.generate([PROMPTS[2]], SamplingParams(temperature=0.0, max_tokens=10, stop_token_ids=[tok]))[0]
    assert r.finish_reason == "stop" and r.output_ids[-1] == tok and len(r.output_ids) == k + 1
    assert out.finish_reason == "length" and len(out.output_ids) == 10


def test_abort_frees_blocks(model):
    e = _engine(model)
    used0 = e.sched.used_blocks()
    r = e.add_request(PROMPTS[0], SamplingParams(max_tokens=50, ignore_eos=True))
    e.step()
    assert e.sched.used_blocks() > used0
    e.abort(r.id)
    assert r.finish_reason == "abort" and not e.has_work()


def test_reference_sampler_truncation():
    torch.manual_seed(0)
    lg = torch.randn(4, 1000)
    t, _ = ref.sample(lg.clone(), torch.tensor([1.0] * 4), torch.tensor([5, 0, 1, 0]), torch.tensor([1.0, 0.3, 1.0, 1.0]),
                      torch.arange(4), torch.zeros(4, dtype=torch.int64))
    assert lg[0, t[0]] >= torch.topk(lg[0], 5).values[-1]
    assert t[2] == torch.argmax(lg[2])
    probs = torch.softmax(lg[1], 0)
    order = torch.argsort(probs, descending=True)
    cs = torch.cumsum(probs[order], 0)
    nucleus = set(order[: int((cs < 0.3).sum()) + 1].tolist())
    assert int(t[1]) in nucleus


def test_embedding_engine_packing_order_and_truncation():
    from nv_genai_amd.engine.embed_engine import EmbeddingEngine

    e = EmbeddingEngine("encoder-tiny", device="cpu", max_batch_tokens=64)
    texts = ["short", "a much longer piece of text " * 5, "mid length text here"]
    together = e.embed(texts)
    alone = torch.cat([e.embed([t]) for t in texts])
    assert torch.allclose(together, alone, atol=1e-4)
    assert torch.allclose(together.norm(dim=1), torch.ones(3), atol=1e-4)
    ids = e.tokenize(["x " * 1000], truncate="END")[0]
    assert len(ids) == 512
    with pytest.raises(ValueError):
        e.tokenize(["x " * 1000], truncate="NONE")


def test_pipelined_decode_matches_synchronous(model):
    p = SamplingParams(temperature=0.8, top_p=0.9, max_tokens=12, ignore_eos=True, seed=5)
    a = [r.output_ids for r in _engine(model, async_decode=True).generate(PROMPTS, p)]
    b = [r.output_ids for r in _engine(model, async_decode=False).generate(PROMPTS, p)]
    assert a == b
    # mixed lengths: sequences leave the batch at different steps
    ps = [SamplingParams(temperature=0.0, max_tokens=m, ignore_eos=True) for m in (3, 9, 6)]
    for async_ in (True, False):
        e = _engine(model, async_decode=async_)
        reqs = [e.add_request(pr, pp) for pr, pp in zip(PROMPTS, ps)]
        e.run_until_done(reqs)
        assert [len(r.output_ids) for r in reqs] == [3, 9, 6]
        assert e.sched.used_blocks() == 0 or not e.has_work()


@pytest.mark.parametrize("async_", [True, False])
def test_mixed_prefill_decode_steps_exact(model, async_):
    """Staggered arrivals: later prompts are prefilled inside steps that also decode the
    running ones (mixed steps); greedy outputs equal the unmixed engine's."""
    p = SamplingParams(temperature=0.0, max_tokens=12, ignore_eos=True)
    outs = []
    for mixed, align, mn in ((0, 1, 0), (40, 1, 0), (40, 16, 0), (64, 16, 100)):
        e = _engine(model, mixed_prefill_tokens=mixed, async_decode=async_, token_alignment=align,
                    mixed_min_tokens=mn, mixed_max_wait=3)
        reqs = [e.add_request(PROMPTS[0], p)]
        for i, pr in enumerate(PROMPTS[1:] + [[5, 6, 7] * 30]):
            for _ in range(3):
                e.step()
            reqs.append(e.add_request(pr, p))
        e.run_until_done(reqs)
        outs.append([r.output_ids for r in reqs])
        if mixed:
            assert e.stats["mixed_steps"] > 0
        else:
            assert e.stats["mixed_steps"] == 0
    assert outs[0] == outs[1] == outs[2] == outs[3]


@pytest.mark.parametrize("temp", [0.0, 1.0])
def test_json_object_output_is_valid_json(model, temp):
    """response_format=json_object: the grammar mask (csrc/runtime/json_grammar.cpp) makes
    even a random-weight model emit one syntactically valid JSON object, then stop."""
    import json

    e = _engine(model)
    p = SamplingParams(temperature=temp, max_tokens=120, response_format="json_object", seed=11)
    outs = e.generate([PROMPTS[0], PROMPTS[1]], p)
    for r in outs:
        if r.finish_reason == "stop":
            obj = json.loads(r.text)
            assert isinstance(obj, dict)
        else:   # cut by max_tokens: still a valid JSON prefix
            from nv_genai_amd._native import rt

            assert r.finish_reason == "length" and rt.JsonState(True).feed(r.text)
    assert not e.has_work()


def test_json_grammar_mask_semantics():
    from nv_genai_amd._native import rt

    toks = [b"{", b"}", b'"a"', b":", b" 1", b"x", b"", b'{"', b"[1]"]
    g = rt.JsonGrammar(toks, [100])
    import numpy as np

    m = np.zeros(101, dtype=np.uint8)
    s = rt.JsonState(True)
    g.fill_mask(s, m)
    # ids past the tokenizer fold onto it (i % 9), as the detokenizer does
    assert [i for i in range(9) if m[i]] == [0, 7] and m[100] == 0   # object start only
    for t in (0, 2, 3, 4):
        assert g.advance(s, t)
    g.fill_mask(s, m)
    assert m[1] == 1 and m[5] == 0 and m[100] == 0
    assert g.advance(s, 1) and s.done
    g.fill_mask(s, m)
    assert [i for i in range(101) if m[i]] == [100]         # complete: only the stop token


@pytest.mark.parametrize("model", ["llama-tiny", "gemma-tiny"])
def test_fp8_w8a8_model_close_to_bf16(model):
    """W8A8 mode (LlamaModel.quantize_fp8): per-channel FP8 weights, per-row FP8 activations;
    the forward stays close to the bf16 model and the engine serves it (SwiGLU and Gemma's
    GeGLU down projection both go through the FP8 GEMM)."""
    from nv_genai_amd.models.config import llama_config
    from nv_genai_amd.models.llama import LlamaModel
    from nv_genai_amd.parallel.dist import ParallelContext
    from nv_genai_amd.training.functional import llama_hidden  # noqa: F401  (bf16 path import)

    cfg = llama_config(model)
    sd = LlamaModel(cfg, "cpu", pctx=ParallelContext(), seed=4).state_dict()
    outs = {}
    for fp8 in (False, True):
        m = LlamaModel(cfg, "cpu", pctx=ParallelContext(), weights=sd, fp8=fp8)
        assert m.fp8 == fp8 and ("wqkv" in m.layers[0]) != fp8
        e = LLMEngine(EngineConfig(model=model, max_num_seqs=4, max_batched_tokens=256, max_model_len=512,
                                   kv_cache_blocks=32), device="cpu", model=m, model_cfg=cfg)
        cap = {}
        orig = e._sample

        def sample(logits, n, cap=cap, orig=orig):
            cap.setdefault("lg", logits[:n].float().clone())
            return orig(logits, n)
        e._sample = sample
        r = e.generate([PROMPTS[0]], SamplingParams(temperature=0.0, max_tokens=4, ignore_eos=True))[0]
        outs[fp8] = (cap["lg"], r.output_ids)
    a, b = outs[False][0], outs[True][0]
    assert float((a - b).norm() / a.norm()) < 0.15
    assert len(outs[True][1]) == 4


def test_prefill_worklist_plan_covers_every_row_once():
    """plan_prefill_items + the work-list semantics (reference) reproduce paged prefill
    attention on the prefill sequences of a mixed step and leave the decode rows alone;
    items are ordered longest key range first."""
    import numpy as np

    from nv_genai_amd import ops
    from nv_genai_amd.ops import reference as ref

    torch.manual_seed(0)
    Hq, Hkv, D = 8, 2, 128
    nd = 3
    ctxs = [50, 7, 130] + [200, 65, 1, 129]
    qls = [1] * nd + [200, 30, 1, 129]
    pages = [(c + 63) // 64 for c in ctxs]
    nb = sum(pages)
    kc = torch.randn(nb, Hkv, 64, D)
    vc = torch.randn(nb, Hkv, D, 64)
    bt = torch.zeros(len(ctxs), max(pages), dtype=torch.int32)
    k = 0
    for i, p in enumerate(pages):
        bt[i, :p] = torch.arange(k, k + p)
        k += p
    cu = np.concatenate([[0], np.cumsum(qls)]).astype(np.int32)
    q = torch.randn(int(cu[-1]), Hq * D)
    items = ops.plan_prefill_items(cu, np.array(ctxs), nd, len(ctxs), Hq, Hkv)
    rw = ops.prefill_rows_per_block(Hq, Hkv)
    assert rw == 32 and len(items) == 7 + 1 + 1 + 5     # 32-row blocks of 200, 30, 1, 129 rows
    out = torch.full((int(cu[-1]), Hq * D), 5.0)
    ref.prefill_attention_worklist(q, kc, vc, bt, torch.from_numpy(cu), torch.tensor(ctxs), Hq, Hkv, D ** -0.5,
                                   torch.from_numpy(items), torch.tensor([len(items)]), out=out, rw=rw)
    want = ref.prefill_attention_paged(q[nd:], kc, vc, bt[nd:], torch.from_numpy(cu[nd:] - cu[nd]),
                                       torch.tensor(ctxs[nd:]), Hq, Hkv, D, D ** -0.5)
    assert torch.allclose(out[nd:], want, atol=1e-5)
    assert bool((out[:nd] == 5.0).all())
    tiles = [(ctxs[b] - qls[b] + min(qls[b] - 1, qb * rw + rw - 1)) // 64 + 1 for b, qb in items.tolist()]
    assert tiles == sorted(tiles, reverse=True)


@pytest.mark.parametrize("async_,head_dim", [(True, 128), (False, 128), (True, 64)])
def test_graph_step_layout_matches_eager(async_, head_dim):
    """The graph-captured prefill / mixed step body (engine mixed_graphs, run without capture
    on CPU: graph_eager) — token rows padded to the bucket, decode rows past the step's own
    skipped, prefill attention from the host work list over absolute rows, S sampling rows —
    generates exactly the eager steps' tokens and log-probabilities."""
    from nv_genai_amd.models.config import llama_config
    from nv_genai_amd.models.llama import LlamaModel
    from nv_genai_amd.parallel.dist import ParallelContext

    cfg = llama_config("llama-tiny", head_dim=head_dim)   # 128: 32x32 work-list kernel, 64: 16x16
    m = LlamaModel(cfg, "cpu", dtype=torch.float32, pctx=ParallelContext(), seed=5)
    prompts = [[3, 4, 5, 6] * 25, [7, 8] * 40, [9] * 5, [11, 12, 13] * 30, [2] * 70]
    p = SamplingParams(temperature=0.0, max_tokens=7, ignore_eos=True, logprobs=True)
    outs = {}
    for graphs in (False, True):
        e = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=8, max_batched_tokens=160, max_model_len=512,
                                   kv_cache_blocks=64, mixed_prefill_tokens=64, token_alignment=32,
                                   async_decode=async_, mixed_graphs=graphs, graph_eager=graphs,
                                   graph_token_step=32), device="cpu", model=m, model_cfg=cfg)
        assert e._mg_ok == graphs
        if graphs:
            assert e._pf_impl == (2 if head_dim == 128 else 1)
        calls = []
        if graphs:
            orig = e._graph_step
            e._graph_step = lambda key, *a, **k: (calls.append(key), orig(key, *a, **k))[1]
        reqs = [e.add_request(pr, p) for pr in prompts[:3]]
        e.step()
        reqs += [e.add_request(pr, p) for pr in prompts[3:]]   # arrive while the first ones decode
        e.run_until_done(reqs)
        outs[graphs] = [(r.output_ids, r.logprobs) for r in reqs]
        if graphs:
            assert calls and any(k[1] > 0 for k in calls)       # mixed steps went through the body
            assert all(k[0] % 32 == 0 for k in calls)
    for (a, la), (b, lb) in zip(outs[False], outs[True]):
        assert a == b
        assert torch.allclose(torch.tensor(la), torch.tensor(lb), atol=1e-4)


def test_graph_key_token_bucket_covers_decode_bucket():
    """Fine token buckets: a mostly-decode step may round to fewer tokens than its decode-row
    bucket; the key's token bucket is raised so the captured decode launch's rows exist."""
    e = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=64, max_batched_tokens=512, max_model_len=512,
                               kv_cache_blocks=64, mixed_prefill_tokens=256, mixed_graphs=True, graph_eager=True,
                               graph_token_step=32), device="cpu")
    assert e._mg_ok
    tb, ndb = e._graph_key(40, 40, 39)     # 39 decode rows + 1 prompt token
    assert ndb == 64 and tb >= ndb and tb % 32 == 0
    assert e._graph_key(10, 100, 0) == (128, 0)


def test_linear_rows_split_matches_matmul():
    """ops.linear_rows_split (the o / down GEMM of full mixed steps, rows cut at a multiple of
    4,096) writes the same rows as one x @ W^T."""
    from nv_genai_amd import ops

    g = torch.Generator().manual_seed(0)
    w = torch.randn(48, 96, generator=g)
    for m, split in ((300, 256), (256, 256), (100, 256), (513, 512), (70, 0)):
        x = torch.randn(m, 96, generator=g)
        out = ops.linear_rows_split(x, w, split=split)
        assert out.shape == (m, 48)
        assert torch.allclose(out, x @ w.t(), atol=1e-5)
    buf = torch.empty(300, 48)
    x = torch.randn(300, 96, generator=g)
    assert ops.linear_rows_split(x, w, buf, 256).data_ptr() == buf.data_ptr()


def test_gemm_operand_guard_rejects_strided_weight_views():
    """ops.linear / linear_rows_split refuse the permuted split-K weight view that faulted the
    library GEMM in the round-3 probe; plain weights pass and match x @ w^T."""
    import pytest
    import torch

    from nv_genai_amd import ops

    x = torch.randn(8, 64)
    w = torch.randn(32, 64)
    assert torch.allclose(ops.linear(x, w), x @ w.t())
    assert torch.allclose(ops.linear_rows_split(x, w, split=4), x @ w.t())
    batched = w.t().reshape(4, 16, 32).permute(0, 2, 1)            # the probe's [s, N, K/s] split-K view
    with pytest.raises(ValueError, match="contiguous row-major"):
        ops.linear(x[:, :16], batched)
    with pytest.raises(ValueError):
        ops.linear(x, w.t().contiguous().t())                      # column-major storage
    with pytest.raises(ValueError):
        ops.linear_rows_split(x, w[:, ::2], split=4)


def test_decode_shape_ops_cpu_fallbacks_match_fp32():
    """The CPU paths of the decode-shape ops (what the engine runs without a GPU) agree with a
    plain fp32 formulation: GEMV epilogues, split-K SwiGLU, split-K add + RMSNorm."""
    from nv_genai_amd import ops

    g = torch.Generator().manual_seed(0)
    x = torch.randn(3, 64, generator=g).to(torch.bfloat16)
    w = (torch.randn(20, 64, generator=g) * 0.1).to(torch.bfloat16)
    y = x.float() @ w.float().t()
    assert torch.allclose(ops.gemv(x, w, 1), y, atol=1e-5)
    assert torch.allclose(ops.gemv(x, w, 0).float(), y, atol=2e-2, rtol=1e-2)
    sw = torch.nn.functional.silu(y[:, :10]) * y[:, 10:]
    assert torch.allclose(ops.gemv(x, w, 2).float(), sw, atol=2e-2, rtol=1e-2)
    P = torch.randn(3, 5, 16, generator=g)
    s = P.sum(0)
    assert torch.allclose(ops.splitk_swiglu(P).float(), torch.nn.functional.silu(s[:, :8]) * s[:, 8:],
                          atol=3e-2, rtol=1e-2)
    resid = torch.randn(5, 16, generator=g).to(torch.bfloat16)
    nw = torch.ones(16, dtype=torch.bfloat16)
    r0 = resid.float() + s
    out = ops.splitk_add_rmsnorm(resid, P, nw, 1e-5)
    assert torch.allclose(resid.float(), r0, atol=3e-2, rtol=1e-2)
    assert torch.allclose(out.float(), ref.rmsnorm(resid.float(), nw.float(), 1e-5), atol=3e-2, rtol=1e-2)
