"""Property-based tests (hypothesis), SURVEY.md §4 item 1: the native scheduler / paged-KV
block manager under random operation sequences (CPU), IVF recall against exact search (CPU),
and on the GPU the top-k kernel's exactness with ties and the sampling kernel's distribution."""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, example, given, settings
from hypothesis import strategies as st

from nv_genai_amd._native import rt

BS = 64


def _bufs(T=2048, S=16, MB=32):
    z = lambda n, dt=np.int32: np.zeros(n, dtype=dt)  # noqa: E731
    return (z(T), z(T), z(T), z(S + 1), z(S), np.zeros((S, MB), dtype=np.int32), z(S, np.int64), z(S))


ops_strategy = st.lists(
    st.one_of(
        st.tuples(st.just("add"), st.integers(1, 300), st.integers(1, 40)),
        st.tuples(st.just("step"), st.integers(0, 0), st.integers(0, 0)),
        st.tuples(st.just("finish"), st.integers(0, 50), st.integers(0, 0)),
        st.tuples(st.just("fork"), st.integers(0, 50), st.integers(0, 0)),
    ), min_size=1, max_size=60)


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(ops=ops_strategy, nblocks=st.integers(8, 48), prefix=st.booleans(), mixed=st.sampled_from([0, 128]))
def test_scheduler_invariants(ops, nblocks, prefix, mixed):
    """Whatever the interleaving of arrivals, steps, finishes and beam forks:
    * no two tokens of one step write the same KV slot, and every slot lies in a block of the
      row's own block table;
    * a slot written in a step is never inside a block another running sequence reads
      (copy-on-fork / prefix sharing never lets a write hit a shared page);
    * used + free == total, and everything is returned once all sequences finish."""
    s = rt.Scheduler(nblocks, BS, 16, 512, 2048, prefix)
    s.set_mixed_prefill_tokens(mixed)
    bufs = _bufs()
    ids, pos, sl, cu, ctx, bt, sid, smp = bufs
    live, nxt = [], 1
    rng = np.random.default_rng(0)
    for op, a, b in ops:
        if op == "add":
            prompt = rng.integers(3, 50, size=a).astype(np.int32).tolist()   # small alphabet: prefix hits
            s.add(nxt, prompt, b)
            live.append(nxt)
            nxt += 1
        elif op == "finish" and live:
            s.finish(live.pop(a % len(live)))
        elif op == "fork" and live:
            p = live[a % len(live)]
            toks = s.tokens(p)
            if toks and toks[-1] >= 0:
                s.fork(p, nxt)
                live.append(nxt)
                nxt += 1
        elif op == "step":
            kind, n, ntok = s.schedule(*bufs)
            if kind == 0:
                continue
            slots = sl[:ntok]
            assert len(set(slots.tolist())) == ntok
            tables = {int(sid[r]): set(bt[r][: (int(ctx[r]) + BS - 1) // BS].tolist()) for r in range(n)}
            for r in range(n):
                own = tables[int(sid[r])]
                for t in range(int(cu[r]), int(cu[r + 1])):
                    blk = int(slots[t]) // BS
                    assert blk in own
                    for o, tb in tables.items():
                        if o != int(sid[r]):
                            assert blk not in tb, "a write lands in a page another sequence reads"
            for r in range(n):
                if smp[r]:
                    s.append_token(int(sid[r]), 7)
        assert s.used_blocks() + s.free_blocks() == s.total_blocks()
    for q in live:
        s.finish(q)
    assert s.used_blocks() == 0 and not s.has_work()


@settings(max_examples=8, deadline=None)
@given(nlist=st.sampled_from([4, 8, 16]), seed=st.integers(0, 1000), k=st.sampled_from([1, 5, 10]))
def test_ivf_recall_property(nlist, seed, k):
    """IVF-Flat: probing every list is exact; probing half of them on clustered data keeps
    recall@k >= 0.9 (the ``GPU_IVF_FLAT`` nlist/nprobe contract of configuration.py:38-47)."""
    from nv_genai_amd.index.flat import FlatIndex
    from nv_genai_amd.index.ivf import IVFFlatIndex

    g = torch.Generator().manual_seed(seed)
    centers = torch.randn(nlist, 32, generator=g)
    X = centers[torch.randint(0, nlist, (2000,), generator=g)] + 0.15 * torch.randn(2000, 32, generator=g)
    Q = X[torch.randint(0, 2000, (20,), generator=g)] + 0.05 * torch.randn(20, 32, generator=g)
    ids = torch.arange(2000)
    flat = FlatIndex(32, "cosine", "cpu")
    flat.add(X, ids)
    ivf = IVFFlatIndex(32, nlist=nlist, nprobe=nlist, metric="cosine", device="cpu")
    ivf.train(X, seed=seed)
    ivf.add(X, ids)
    ve, ie = flat.search(Q, k)
    va, ia = ivf.search(Q, k, nprobe=nlist)
    # exact: the same top-k scores; the same ids wherever the k-th score is not tied with the
    # next one (the two indexes sum the dot products in different orders, so an fp32 tie at
    # the cut can fall either way)
    assert torch.allclose(va, ve, atol=1e-5), (va, ve)
    v1, _ = flat.search(Q, k + 1)
    for qi in range(Q.shape[0]):
        if v1.shape[1] <= k or float(v1[qi, k - 1] - v1[qi, k]) > 1e-5:
            assert set(ia[qi].tolist()) == set(ie[qi].tolist()), qi
    _, ih = ivf.search(Q, k, nprobe=max(1, nlist // 2))
    rec = np.mean([len(set(a.tolist()) & set(e.tolist())) / k for a, e in zip(ih, ie)])
    assert rec >= 0.9, rec


# ----------------------------------------------------------------------------- GPU kernels
@pytest.mark.gpu
@settings(max_examples=25, deadline=None)
@given(rows=st.integers(1, 40), n=st.integers(1, 20000), k=st.integers(1, 128), levels=st.sampled_from([0, 3, 50]))
def test_topk_kernel_exact_with_ties(gpu, rows, n, k, levels):
    """ops.topk (per-segment radix select + merge) returns exactly torch.topk's values, with
    heavy ties when ``levels`` > 0, and indices that point at those values."""
    from nv_genai_amd import ops

    g = torch.Generator(device="cpu").manual_seed(rows * 7919 + n * 31 + k)
    S = torch.randn(rows, n, generator=g)
    if levels:
        S = torch.floor(S * levels) / levels
    S = S.to(gpu)
    v, i = ops.topk(S, k)
    kk = min(k, n)
    v_ref = torch.topk(S.cpu(), kk, dim=1).values
    assert v.shape == (rows, kk)
    assert torch.equal(v.cpu(), v_ref)
    assert torch.equal(torch.gather(S.cpu(), 1, i.cpu().long()), v.cpu())
    assert all(len(set(r.tolist())) == kk for r in i.cpu())


@pytest.mark.gpu
@settings(max_examples=10, deadline=None)
@example(temp=1.0, top_k=5, top_p=0.8, seed=0)   # top-p inside top-k: renormalised
@given(temp=st.sampled_from([0.5, 1.0, 1.5]), top_k=st.sampled_from([0, 5, 20]),
       top_p=st.sampled_from([1.0, 0.8, 0.5]), seed=st.integers(0, 10000))
def test_sampling_kernel_distribution(gpu, temp, top_k, top_p, seed):
    """Draws of the sampling kernel (Gumbel-max over the truncated, tempered distribution,
    counter-based RNG) follow softmax(logits / T) restricted to top-k ∩ top-p: chi-square
    over 16384 independent rows, and no draw outside the kept set."""
    from nv_genai_amd import ops

    V, B = 40, 16384
    g = torch.Generator().manual_seed(seed)
    base = torch.randn(V, generator=g) * 2
    logits = base.expand(B, V).contiguous().to(gpu)
    tok, _ = ops.sample(logits, torch.full((B,), temp, device=gpu),
                        torch.full((B,), top_k, dtype=torch.int32, device=gpu),
                        torch.full((B,), top_p, device=gpu),
                        torch.arange(B, dtype=torch.int64, device=gpu) * 104729 + seed,
                        torch.zeros(B, dtype=torch.int64, device=gpu))
    p = torch.softmax(base / temp, 0).double()
    order = torch.argsort(p, descending=True)
    # TensorRT-LLM / HF semantics: top-k first, then top-p on the renormalised top-k mass
    keep = torch.zeros(V, dtype=torch.bool)
    kmax = top_k if top_k > 0 else V
    mass = float(p[order[:kmax]].sum())
    cum = 0.0
    for j, t in enumerate(order.tolist()[:kmax]):
        if j > 0 and cum >= top_p * mass:
            break
        keep[t] = True
        cum += float(p[t])
    q = torch.where(keep, p, torch.zeros_like(p))
    q /= q.sum()
    counts = torch.bincount(tok.cpu().long(), minlength=V).double()
    assert counts[~keep].sum() == 0, "a draw outside top-k / top-p"
    exp = q * B
    m = exp > 5
    chi2 = float((((counts - exp) ** 2) / exp.clamp_min(1e-9))[m].sum())
    dof = int(m.sum()) - 1
    # a 5-sigma bound on chi-square(dof): mean dof, variance 2 dof
    assert chi2 <= dof + 5 * (2 * max(dof, 1)) ** 0.5 + 5, (chi2, dof)
