"""Fused vector-search kernels on the GPU against fp32 PyTorch references: the MFMA score +
per-block register top-k (flat search, K13) and the batched IVF list scan over (list,
query-chunk) work items (K14)."""
import pytest
import torch

from nv_genai_amd import ops
from nv_genai_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _data(N, D, nq, seed, dev):
    g = torch.Generator(device="cpu").manual_seed(seed)
    X = torch.nn.functional.normalize(torch.randn(N, D, generator=g), dim=1).to(dev, torch.bfloat16)
    Q = torch.nn.functional.normalize(torch.randn(nq, D, generator=g), dim=1).to(dev, torch.bfloat16)
    return X, Q


def _check_topk(v, r, X, Q, bias, scale, k):
    """Returned scores are the exact scores of the returned rows, sorted, and no row outside
    the result scores above the k-th (ties aside)."""
    S = ref.score(Q, X, bias, scale)                       # fp32 reference [nq, N]
    rv, _ = torch.topk(S, k, dim=1)
    assert v.shape == (Q.shape[0], k) and r.shape == (Q.shape[0], k)
    fin = torch.isfinite(rv)
    assert torch.equal(torch.isfinite(v), fin)
    assert torch.allclose(v[fin], rv[fin], atol=2e-3, rtol=1e-3)
    assert bool((r[~fin] == -1).all()) and bool((r[fin] >= 0).all())
    got = torch.gather(S, 1, r.clamp_min(0))
    assert torch.allclose(got[fin], v[fin], atol=2e-3, rtol=1e-3)
    assert bool((v[:, :-1] >= v[:, 1:]).all())
    for row in r.tolist():                                  # distinct rows
        live = [x for x in row if x >= 0]
        assert len(set(live)) == len(live)


@pytest.mark.parametrize("N,D,nq,k", [(1000, 128, 1, 4), (100_003, 1024, 1, 4), (100_003, 1024, 8, 8),
                                      (50_000, 384, 33, 16), (70_001, 1024, 64, 4), (70_001, 1024, 100, 8),
                                      (3, 128, 5, 4), (20_000, 1024, 17, 1),
                                      # LDS-DMA form: 256- and 512-dim chunks, partial last tile
                                      (30_011, 768, 16, 16), (20_000, 2048, 3, 4), (5_000, 256, 2, 4),
                                      (777, 1024, 16, 8)])
def test_search_topk_matches_reference(gpu, N, D, nq, k):
    X, Q = _data(N, D, nq, N + nq, gpu)
    bias = torch.zeros(N, device=gpu)
    bias[::7] = float("-inf")                                # tombstones
    v, r = ops.search_topk(Q, X, bias, 1.0, k)
    _check_topk(v, r, X, Q, bias, 1.0, min(k, N))


def test_search_topk_l2_bias_and_no_bias(gpu):
    X, Q = _data(30_000, 256, 12, 5, gpu)
    bias = -ops.row_sqnorm(X)
    v, r = ops.search_topk(Q, X, bias, 2.0, 8)
    _check_topk(v, r, X, Q, bias, 2.0, 8)
    v, r = ops.search_topk(Q, X, None, 1.0, 8)
    _check_topk(v, r, X, Q, None, 1.0, 8)


def test_search_topk_large_k_falls_back(gpu):
    X, Q = _data(10_000, 128, 4, 9, gpu)
    v, r = ops.search_topk(Q, X, None, 1.0, 50)                # beyond the register lists
    _check_topk(v, r, X, Q, None, 1.0, 50)


@pytest.mark.parametrize("nq,nprobe,k", [(1, 16, 4), (8, 16, 8), (64, 16, 4), (70, 5, 8), (20, 16, 16)])
def test_ivf_scan_matches_reference(gpu, nq, nprobe, k):
    N, D, nlist = 60_000, 256, 64
    X, Q = _data(N, D, nq, 11 + nq, gpu)
    # list-sorted slab with uneven lists, some empty
    sizes = torch.randint(0, 2 * N // nlist, (nlist,), generator=torch.Generator().manual_seed(1))
    sizes[3] = 0
    sizes[10] = 0
    off = torch.cat([torch.zeros(1, dtype=torch.int64), sizes.cumsum(0)])
    Xs = X[: int(off[-1])].contiguous()
    beg, end = off[:-1].to(gpu), off[1:].to(gpu)
    bias = torch.zeros(Xs.shape[0], device=gpu)
    bias[::5] = float("-inf")
    g = torch.Generator().manual_seed(nq)
    probes = torch.stack([torch.randperm(nlist, generator=g)[:nprobe] for _ in range(nq)]).to(gpu)
    probes[0, 0] = 3                                            # an empty list is probed
    v, r = ops.ivf_search_topk(Q, Xs, bias, 1.0, probes, beg, end, int(sizes.max()), k)
    rv, rr = ref.ivf_search_topk(Q, Xs, bias, 1.0, probes, beg, end, k)
    fin = torch.isfinite(rv)
    assert torch.equal(torch.isfinite(v), fin)
    assert torch.allclose(v[fin], rv[fin], atol=2e-3, rtol=1e-3)
    S = ref.score(Q, Xs, bias, 1.0)
    assert torch.allclose(torch.gather(S, 1, r.clamp_min(0))[fin], v[fin], atol=2e-3, rtol=1e-3)
    assert bool((r[~fin] == -1).all())


def test_ivf_scan_splits_past_item_limit(gpu):
    """nlist 4,096 with 1,100 queries is 4,096 x 18 = 73,728 (list, query-chunk) items, past
    the scan launch's 65,535: the queries run in two sub-batches and still match the reference."""
    N, D, nlist, nq, nprobe, k = 40_000, 128, 4096, 1100, 4, 4
    X, Q = _data(N, D, nq, 23, gpu)
    sizes = torch.randint(0, 2 * N // nlist, (nlist,), generator=torch.Generator().manual_seed(2))
    off = torch.cat([torch.zeros(1, dtype=torch.int64), sizes.cumsum(0)])
    Xs = X[: int(off[-1])].contiguous()
    beg, end = off[:-1].to(gpu), off[1:].to(gpu)
    g = torch.Generator().manual_seed(5)
    probes = torch.stack([torch.randperm(nlist, generator=g)[:nprobe] for _ in range(nq)]).to(gpu)
    assert nlist * -(-nq // 64) > ops.IVF_MAX_ITEMS
    v, r = ops.ivf_search_topk(Q, Xs, None, 1.0, probes, beg, end, int(sizes.max()), k)
    rv, rr = ref.ivf_search_topk(Q, Xs, None, 1.0, probes, beg, end, k)
    fin = torch.isfinite(rv)
    assert v.shape == (nq, k) and torch.equal(torch.isfinite(v), fin)
    assert torch.allclose(v[fin], rv[fin], atol=2e-3, rtol=1e-3)


def test_ivf_index_recall_vs_flat_nlist64_nprobe16(gpu):
    """The reference's GPU_IVF_FLAT setting (nlist 64, nprobe 16) on clustered data: batched
    IVF search finds >= 95% of the flat index's top-10 (RetrievalAugmentedGeneration/common/
    utils.py:198-203)."""
    from nv_genai_amd.index.flat import FlatIndex
    from nv_genai_amd.index.ivf import IVFFlatIndex

    g = torch.Generator().manual_seed(7)
    centers = torch.randn(200, 512, generator=g)
    X = centers[torch.randint(0, 200, (200_000,), generator=g)] + 0.4 * torch.randn(200_000, 512, generator=g)
    Q = X[torch.randint(0, 200_000, (48,), generator=g)] + 0.1 * torch.randn(48, 512, generator=g)
    ids = torch.arange(200_000) * 3 + 1
    flat = FlatIndex(512, "cosine", gpu, capacity=200_000)
    flat.add(X, ids)
    ivf = IVFFlatIndex(512, nlist=64, nprobe=16, metric="cosine", device=gpu)
    ivf.train(X[:50_000])
    ivf.add(X, ids)
    assert len(ivf) == 200_000
    fv, fi = flat.search(Q, 10)
    iv, ii = ivf.search(Q, 10)
    recall = sum(len(set(a) & set(b)) for a, b in zip(ii.tolist(), fi.tolist())) / fi.numel()
    assert recall >= 0.95, recall
    assert ivf.remove(ii[:, 0].tolist()) == len(set(ii[:, 0].tolist()))
    assert len(ivf) == 200_000 - len(set(ii[:, 0].tolist()))
    _, ii2 = ivf.search(Q, 10)
    assert not set(ii[:, 0].tolist()) & set(ii2.reshape(-1).tolist())
