"""Beam search (engine/beam.py) on CPU: copy-on-fork paged KV against a brute-force beam
search that recomputes every hypothesis from scratch, stop-token hypotheses, length penalty,
block accounting, and the native scheduler's fork."""
import pytest
import torch

from nv_genai_amd._native import rt
from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine, SamplingParams
from nv_genai_amd.training.functional import llama_hidden


@pytest.fixture(scope="module")
def model():
    from nv_genai_amd.models.config import llama_config
    from nv_genai_amd.models.llama import LlamaModel
    from nv_genai_amd.parallel.dist import ParallelContext

    return LlamaModel(llama_config("llama-tiny"), "cpu", pctx=ParallelContext(), seed=5)


def _engine(model, **kw):
    cfg = dict(model="llama-tiny", max_num_seqs=16, max_batched_tokens=256, max_model_len=512,
               kv_cache_blocks=96)
    cfg.update(kw)
    return LLMEngine(EngineConfig(**cfg), device="cpu", model=model)


def _next_logprobs(model, seqs):
    with torch.no_grad():
        out = []
        for s in seqs:
            h = llama_hidden(model, torch.tensor([s]))[0, -1:]
            out.append(torch.log_softmax(model.logits(h).float(), -1)[0])
        return out


def _brute_beam(model, prompt, width, steps, lp=1.0, stop=()):
    beams = [(0.0, [])]
    hyps = []
    for cur in range(1, steps + 1):
        lps = _next_logprobs(model, [prompt + b for _, b in beams])
        cands = []
        for (score, toks), l in zip(beams, lps):
            v, i = l.topk(2 * width)
            cands += [(score + float(a), toks, int(t)) for a, t in zip(v, i)]
        cands.sort(key=lambda c: -c[0])
        nxt = []
        for rank, (score, toks, t) in enumerate(cands):
            if t in stop:
                if rank < width:
                    hyps.append((score / (cur ** lp), toks + [t]))
                continue
            nxt.append((score, toks + [t]))
            if len(nxt) == width:
                break
        hyps.sort(key=lambda h: -h[0])
        hyps = hyps[:width]
        if len(hyps) >= width and nxt[0][0] / cur ** lp <= hyps[-1][0]:
            return hyps
        beams = nxt
    hyps += [(s / (steps ** lp), t) for s, t in beams]
    hyps.sort(key=lambda h: -h[0])
    return hyps[:width]


def _rescore(model, prompt, toks):
    """Sum of the log-probs of ``toks`` after ``prompt`` from one full causal forward."""
    with torch.no_grad():
        h = llama_hidden(model, torch.tensor([prompt + toks]))[0, len(prompt) - 1: -1]
        lp = torch.log_softmax(model.logits(h).float(), -1)
        return float(lp.gather(1, torch.tensor(toks)[:, None]).sum())


# prompt lengths straddle the 64-token page: 61 + 8 generated crosses a page boundary
# while beams fork (partial-page copies), 130 shares two full pages between forks.
# bf16 rounding differs between the paged kernels and the padded reference, so near-tied
# beams may swap; the best beam must match and every returned beam must score (recomputed
# from scratch, which checks the forked KV) what the engine says it scores.
@pytest.mark.parametrize("plen,width", [(61, 3), (130, 4)])
def test_beam_matches_bruteforce(model, plen, width):
    prompt = [(7 * i + 3) % 500 + 10 for i in range(plen)]
    e = _engine(model)
    used0 = e.sched.used_blocks()
    r = e.generate([prompt], SamplingParams(beam_width=width, max_tokens=8, ignore_eos=True))[0]
    ref = _brute_beam(model, prompt, width, 8)
    assert r.finished and r.finish_reason == "length" and len(r.beams) == width
    assert r.output_ids == ref[0][1]
    for (s, toks, _), (rs, _) in zip(r.beams, ref):
        assert abs(s - rs) < 3e-2
        assert abs(s * len(toks) - _rescore(model, prompt, toks)) < 0.15
    assert len({tuple(b[1]) for b in r.beams}) == width
    assert e.sched.used_blocks() == used0 and not e._beam_of and not e.has_work()


def test_beam_stop_token_and_length_penalty(model):
    prompt = [(11 * i + 5) % 400 + 20 for i in range(70)]
    e = _engine(model)
    free = e.generate([prompt], SamplingParams(beam_width=2, max_tokens=6, ignore_eos=True))[0]
    stop = free.output_ids[2]
    for lp in (1.0, 0.0):
        r = e.generate([prompt], SamplingParams(beam_width=2, max_tokens=6, stop_token_ids=[stop],
                                                length_penalty=lp))[0]
        ref = _brute_beam(model, prompt, 2, 6, lp=lp, stop=(stop,))
        assert r.output_ids == ref[0][1] and abs(r.beams[0][0] - ref[0][0]) < 3e-2
        assert r.finish_reason == ("stop" if r.output_ids[-1] == stop else "length")


def test_beam_rides_with_sampled_requests(model):
    """A beam group and greedy requests share the continuous batch; greedy output is unchanged."""
    p1 = [5, 6, 7] * 30
    g = SamplingParams(temperature=0.0, max_tokens=7, ignore_eos=True)
    solo = _engine(model).generate([p1], g)[0].output_ids
    e = _engine(model)
    a = e.add_request(p1, g)
    b = e.add_request([9, 10] * 40, SamplingParams(beam_width=3, max_tokens=7, ignore_eos=True))
    e.run_until_done([a, b])
    assert a.output_ids == solo and b.finished and len(b.output_ids) == 7


def test_beam_abort_frees_everything(model):
    e = _engine(model)
    used0 = e.sched.used_blocks()
    r = e.add_request([3] * 90, SamplingParams(beam_width=4, max_tokens=50, ignore_eos=True))
    for _ in range(4):
        e.step()
    assert len(e._beam_of) == 4
    e.abort(r.id)
    assert r.finish_reason == "abort" and not e._beam_of
    assert e.sched.used_blocks() == used0 and not e.has_work()


def test_scheduler_fork_shares_full_pages():
    s = rt.Scheduler(16, 64, 8, 512, 1024, True)
    s.add(1, list(range(100)), 20)
    ids, pos, sl, cu, ctx = (torch.zeros(512, dtype=torch.int32).numpy() for _ in range(5))
    bt = torch.zeros(8, 16, dtype=torch.int32).numpy()
    sid = torch.zeros(8, dtype=torch.int64).numpy()
    smp = torch.zeros(8, dtype=torch.int32).numpy()
    s.schedule(ids, pos, sl, cu, ctx, bt, sid, smp)
    used = s.used_blocks()
    src, dst = s.fork(1, 2)
    assert src >= 0 and dst >= 0 and src != dst       # 100 % 64 != 0: last page copied
    assert s.used_blocks() == used + 1                # the full page is shared, not copied
    assert s.tokens(2) == s.tokens(1)
    s.finish(1)
    assert s.used_blocks() == used                    # shared page still held by the child
    s.finish(2)
    assert s.used_blocks() == 0


def test_frequency_presence_penalties_greedy(model):
    """Greedy with count penalties equals greedy over logits minus f*count + p*[count>0]:
    checked step by step against the padded reference forward."""
    prompt = [4, 5, 6] * 22
    f, p = 0.7, 0.9
    r = _engine(model).generate([prompt], SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True,
                                                         frequency_penalty=f, presence_penalty=p))[0]
    out = []
    for _ in range(8):
        lg = _next_logprobs(model, [prompt + out])[0]
        cnt = torch.bincount(torch.tensor(out, dtype=torch.int64), minlength=lg.numel()) if out else 0
        out.append(int((lg - f * cnt - p * (cnt > 0 if out else 0)).argmax()))
    assert r.output_ids == out
