"""Numerics of every gfx950 HIP kernel against the plain-PyTorch fp32 reference of the same op."""
import math

import pytest
import torch

from nv_genai_amd import ops
from nv_genai_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _bf(*shape, dev, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(torch.bfloat16)


def _close(a, b, atol, rtol=0.0):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    lim = atol + rtol * b.abs().max().item()
    assert err <= lim, f"max err {err} > {lim}"


def _close_rows(a, b, width=None, rel=1e-2, peak=2e-2):
    """Relative error per output vector (every row, or every ``width``-wide head slice of a
    row): ||a - b|| <= rel * ||b|| for each vector, and max |a - b| <= peak * max |b| overall.
    Attention outputs shrink like sqrt(e / ctx) at long context, so an absolute bound would
    stop seeing errors confined to part of a sequence; a per-vector relative bound does not."""
    a, b = a.float().cpu(), b.float().cpu()
    assert a.shape == b.shape
    if width is not None:
        a, b = a.reshape(-1, width), b.reshape(-1, width)
    else:
        a, b = a.reshape(a.shape[0], -1), b.reshape(b.shape[0], -1)
    rn = b.norm(dim=1)
    live = rn > 0
    en = (a - b).norm(dim=1)
    assert bool((en[~live] == 0).all()), "rows with a zero reference must be exactly zero"
    worst = (en[live] / rn[live]).max().item() if bool(live.any()) else 0.0
    assert worst <= rel, f"worst per-vector relative error {worst:.4g} > {rel}"
    pk = (a - b).abs().max().item()
    assert pk <= peak * b.abs().max().item() + 1e-6, f"max abs err {pk:.4g} > {peak} x max|ref|"


@pytest.mark.parametrize("H", [768, 1024, 2048, 3072, 4096, 5120, 6144, 8192])
def test_rmsnorm(gpu, H):
    torch.manual_seed(0)
    x, w = _bf(37, H, dev=gpu), _bf(H, dev=gpu)
    _close_rows(ops.rmsnorm(x, w, 1e-5), ref.rmsnorm(x.cpu().float(), w.cpu().float(), 1e-5))
    r, d = _bf(37, H, dev=gpu), _bf(37, H, dev=gpu)
    r_ref = r.cpu().clone()
    y = ops.add_rmsnorm(r, d, w, 1e-5)
    y_ref = ref.add_rmsnorm(r_ref, d.cpu(), w.cpu(), 1e-5)
    _close_rows(r, r_ref)
    _close_rows(y, y_ref)


def test_layernorm_gelu_silu(gpu):
    torch.manual_seed(1)
    x, r, g, b = _bf(33, 1024, dev=gpu), _bf(33, 1024, dev=gpu), _bf(1024, dev=gpu), _bf(1024, dev=gpu)
    _close_rows(ops.layernorm(x, g, b, 1e-12, resid=r), ref.layernorm(x.cpu(), g.cpu(), b.cpu(), 1e-12, r.cpu()))
    h = _bf(17, 4096, dev=gpu)
    bias = _bf(4096, dev=gpu)
    h_ref = h.cpu().clone()
    ops.bias_gelu_(h, bias)
    ref.bias_gelu_(h_ref, bias.cpu())
    _close_rows(h, h_ref)
    gu = _bf(19, 2 * 14336, dev=gpu)
    _close_rows(ops.silu_mul(gu), ref.silu_mul(gu.cpu()))


def _make_cache(nb, Hkv, D, dev):
    kc = _bf(nb, Hkv, 64, D, dev=dev)
    vc = _bf(nb, Hkv, D, 64, dev=dev)
    return kc, vc


@pytest.mark.parametrize("vnt", [0, 1, 2])
@pytest.mark.parametrize("Hq,Hkv,D,T", [(32, 8, 128, 70), (32, 8, 128, 7), (32, 8, 128, 300), (4, 2, 64, 130)])
def test_rope_cache(gpu, kernel_form, Hq, Hkv, D, T, vnt):
    """per-token kernel (T < 64) and tiled kernel (T >= 64: LDS-transposed Vt page rows),
    random slots with a padding row (-1); vnt: the non-temporal Vt store form (rope_vnt)."""
    kernel_form("rope_vnt", vnt)
    torch.manual_seed(2)
    qkv = _bf(T, (Hq + 2 * Hkv) * D, dev=gpu)
    pos = torch.randint(0, 4000, (T,), dtype=torch.int32, device=gpu)
    cs = ops.rope_cos_sin(4096, D).to(gpu)
    nb = (T + 63) // 64 + 4
    kc, vc = _make_cache(nb, Hkv, D, gpu)
    slots = torch.randperm(nb * 64, device=gpu)[:T].to(torch.int32)
    slots[5] = -1
    qkv_r, kc_r, vc_r = qkv.cpu().clone(), kc.cpu().clone(), vc.cpu().clone()
    ops.rope_cache_(qkv, pos, cs, slots, kc, vc, Hq, Hkv, D)
    ref.rope_cache_(qkv_r, pos.cpu(), cs.cpu(), slots.cpu(), kc_r, vc_r, Hq, Hkv, D)
    _close_rows(qkv, qkv_r, width=D)
    _close_rows(kc, kc_r, width=D)
    _close(vc, vc_r, 1e-6)


@pytest.mark.parametrize("T", [7, 256, 300])
def test_rope_cache_from_splitk_partials(gpu, T):
    """The RoPE / KV-write kernel fed the qkv projection as K-split fp32 slabs (the skinny
    GEMM's output) writes exactly what the bf16-materialised projection + RoPE writes: q / k
    rotated, v columns, and both caches (per-token and tiled forms)."""
    torch.manual_seed(4)
    Hq, Hkv, D, S = 32, 8, 128, 3
    P = torch.randn(S, T, (Hq + 2 * Hkv) * D, device=gpu)
    pos = torch.randint(0, 4000, (T,), dtype=torch.int32, device=gpu)
    cs = ops.rope_cos_sin(4096, D).to(gpu)
    nb = (T + 63) // 64 + 4
    kc, vc = _make_cache(nb, Hkv, D, gpu)
    slots = torch.randperm(nb * 64, device=gpu)[:T].to(torch.int32)
    slots[3] = -1
    kc2, vc2 = kc.clone(), vc.clone()
    want = ops.splitk_reduce(P)
    ops.rope_cache_(want, pos, cs, slots, kc, vc, Hq, Hkv, D)
    got = torch.full_like(want, float("nan"))
    ops.rope_cache_(got, pos, cs, slots, kc2, vc2, Hq, Hkv, D, partial=ops.PartialSum(P))
    assert torch.equal(got, want) and torch.equal(kc2, kc) and torch.equal(vc2, vc)


def _paged_setup(ctxs, Hkv, D, dev, seed=0):
    torch.manual_seed(seed)
    pages = [(c + 63) // 64 for c in ctxs]
    nb = sum(pages) + 3
    kc, vc = _make_cache(nb, Hkv, D, dev)
    perm = torch.randperm(nb).tolist()
    maxp = max(pages)
    bt = torch.zeros(len(ctxs), maxp, dtype=torch.int32)
    k = 0
    for i, p in enumerate(pages):
        for j in range(p):
            bt[i, j] = perm[k]
            k += 1
    return kc, vc, bt.to(dev)


@pytest.mark.parametrize("aux", ["2", "0"])
@pytest.mark.parametrize("dma", ["1", "2"])
@pytest.mark.parametrize("G", [4, 8])
@pytest.mark.parametrize("ppp", [None, 2, 3])
def test_decode_attention(gpu, G, ppp, dma, aux, kernel_form, monkeypatch):
    """NGA_DECODE_DMA 1: the whole-page LDS-DMA kernel, 2: its half-page ring form (KV loads
    nt, or with NGA_DECODE_DMA_AUX=0 the default cache policy).
    Short, page-edge, long (4096 / 8192) contexts and contexts one key either side of a
    split-K partition boundary (ppp pages of 64 keys per partition), per-head relative error
    against the fp32 reference (computed on the GPU in fp32)."""
    kernel_form("decode_dma", dma)
    kernel_form("decode_dma_aux", aux)
    Hkv, D = 8 if G == 4 else 1, 128
    Hq = Hkv * G
    part = 64 * (ppp or 2)
    ctxs = [1, 63, 64, 65, 700, 3001, 128, 4096, 8192, part - 1, part + 1, 3 * part, 5 * part + 1]
    kc, vc, bt = _paged_setup(ctxs, Hkv, D, gpu)
    B = len(ctxs)
    q = _bf(B, Hq * D, dev=gpu)
    ctx = torch.tensor(ctxs, dtype=torch.int32, device=gpu)
    scale = 1 / math.sqrt(D)
    ws = ops.DecodeWorkspace(B, Hq, Hkv, max(ctxs), gpu, ppp)
    out = ops.decode_attention(q, kc, vc, bt, ctx, Hq, Hkv, max(ctxs), scale, ws=ws)
    o_ref = ref.decode_attention(q.float(), kc, vc, bt, ctx, Hq, Hkv, scale)
    _close_rows(out, o_ref, width=D)


@pytest.mark.parametrize("nt", ["0", "1"])
@pytest.mark.parametrize("D", [128, 256])
def test_decode_attention_register_kernel(gpu, D, nt, kernel_form, monkeypatch):
    """The register decode kernel (NGA_DECODE_DMA=0; head_dim 256 always runs it) with its KV
    loads on the default cache policy or nt (form decode_nt), against the fp32 reference."""
    kernel_form("decode_dma", 0)
    kernel_form("decode_nt", nt)
    Hkv, G = 4, 4
    Hq = Hkv * G
    ctxs = [1, 63, 65, 700, 3001, 4096]
    kc, vc, bt = _paged_setup(ctxs, Hkv, D, gpu, seed=5)
    q = _bf(len(ctxs), Hq * D, dev=gpu)
    ctx = torch.tensor(ctxs, dtype=torch.int32, device=gpu)
    scale = 1 / math.sqrt(D)
    out = ops.decode_attention(q, kc, vc, bt, ctx, Hq, Hkv, max(ctxs), scale)
    o_ref = ref.decode_attention(q.float(), kc, vc, bt, ctx, Hq, Hkv, scale, D=D)
    _close_rows(out, o_ref, width=D)


@pytest.mark.parametrize("dma", ["1", "2"])
def test_decode_attention_empty_rows(gpu, dma, kernel_form, monkeypatch):
    kernel_form("decode_dma", dma)
    Hkv, G, D = 8, 4, 128
    Hq = Hkv * G
    kc, vc, bt = _paged_setup([100, 1], Hkv, D, gpu)
    ctx = torch.tensor([100, 0], dtype=torch.int32, device=gpu)
    q = _bf(2, Hq * D, dev=gpu)
    out = ops.decode_attention(q, kc, vc, bt, ctx, Hq, Hkv, 100, 1 / math.sqrt(D))
    assert torch.isfinite(out.float()).all()
    assert out[1].abs().max().item() == 0.0


def test_prefill_attention_paged(gpu):
    Hkv, G, D = 8, 4, 128
    Hq = Hkv * G
    ctxs = [100, 700, 64, 1, 1500]
    qls = [100, 300, 64, 1, 129]  # second and last: chunked prefill after a cached prefix
    kc, vc, bt = _paged_setup(ctxs, Hkv, D, gpu, seed=3)
    cu = [0]
    for ql in qls:
        cu.append(cu[-1] + ql)
    T = cu[-1]
    q = _bf(T, Hq * D, dev=gpu)
    cu_t = torch.tensor(cu, dtype=torch.int32, device=gpu)
    ctx_t = torch.tensor(ctxs, dtype=torch.int32, device=gpu)
    scale = 1 / math.sqrt(D)
    out = ops.prefill_attention_paged(q, kc, vc, bt, cu_t, ctx_t, Hq, Hkv, D, max(qls), scale)
    o_ref = ref.prefill_attention_paged(q.float(), kc, vc, bt, cu_t, ctx_t, Hq, Hkv, D, scale)
    _close_rows(out, o_ref, width=D)


@pytest.mark.parametrize("Hkv,G,window,causal", [
    (8, 4, 0, True),      # Llama-3-8B: 4 query heads of a GQA group per workgroup
    (2, 8, 0, True),      # Llama-70B-style G = 8: two head groups per KV head
    (4, 1, 0, True),      # MHA: 4 x 32-row blocks of one head per workgroup
    (2, 2, 0, True),      # 2 heads x 2 row blocks
    (1, 3, 0, True),      # odd G: row blocks
    (2, 4, 200, True),    # sliding window (Mistral)
    (2, 4, 0, False),     # bidirectional over the paged cache
])
def test_prefill_attention_v2_layouts(gpu, Hkv, G, window, causal):
    """The 32x32-MFMA paged prefill kernel (attention_prefill_v2.hip) in each of its
    wave-to-(head, row block) layouts, against the fp32 reference: ragged query lengths
    (not multiples of 32), chunked prefill after a cached prefix, single-token rows."""
    D = 128
    Hq = Hkv * G
    ctxs = [100, 700, 64, 1, 1500, 33]
    qls = [100, 300, 64, 1, 1500, 1]
    kc, vc, bt = _paged_setup(ctxs, Hkv, D, gpu, seed=11)
    cu = [0]
    for ql in qls:
        cu.append(cu[-1] + ql)
    q = _bf(cu[-1], Hq * D, dev=gpu)
    cu_t = torch.tensor(cu, dtype=torch.int32, device=gpu)
    ctx_t = torch.tensor(ctxs, dtype=torch.int32, device=gpu)
    scale = 1 / math.sqrt(D)
    o_ref = ref.prefill_attention_paged(q.float(), kc, vc, bt, cu_t, ctx_t, Hq, Hkv, D, scale, causal, window)
    for impl in (2, 3):   # 4-wave, 8-wave split-key
        out = ops.prefill_attention_paged(q, kc, vc, bt, cu_t, ctx_t, Hq, Hkv, D, max(qls), scale,
                                          causal=causal, window=window, impl=impl)
        _close_rows(out, o_ref, width=D)


@pytest.mark.parametrize("impl", [0, 1, 2, 3])
@pytest.mark.parametrize("ctxs,qls,window", [
    ([1200], [940], 0),            # one prompt after a 260-token prefix hit
    ([1200] * 6, [1200] * 6, 0),   # six prompts (the size rule picks the 32x32 kernel)
    ([3000, 64], [2000, 64], 0),   # long + short sequence
    ([1200], [940], 300),          # sliding window
    ([4096, 8192], [4096, 1024], 0),   # long contexts (the last chunk of an 8K prompt)
    ([4160, 127, 129], [4160, 127, 129], 0),   # tile edges: 65 x 64, 64 +- 1 past 2 tiles
])
def test_prefill_attention_kernel_choice(gpu, ctxs, qls, window, impl):
    """Serving-size prefills through the size rule (impl 0) and through each kernel forced,
    against the fp32 reference."""
    Hkv, G, D = 8, 4, 128
    Hq = Hkv * G
    kc, vc, bt = _paged_setup(ctxs, Hkv, D, gpu, seed=13)
    cu = [0]
    for ql in qls:
        cu.append(cu[-1] + ql)
    q = _bf(cu[-1], Hq * D, dev=gpu)
    cu_t = torch.tensor(cu, dtype=torch.int32, device=gpu)
    ctx_t = torch.tensor(ctxs, dtype=torch.int32, device=gpu)
    scale = 1 / math.sqrt(D)
    o_ref = ref.prefill_attention_paged(q.float(), kc, vc, bt, cu_t, ctx_t, Hq, Hkv, D, scale, True, window)
    out = ops.prefill_attention_paged(q, kc, vc, bt, cu_t, ctx_t, Hq, Hkv, D, max(qls), scale,
                                      window=window, impl=impl)
    _close_rows(out, o_ref, width=D)


@pytest.mark.parametrize("D,scales", [(128, (1.0, 1.0)), (128, (3.0, 0.5)), (256, (2.0, 2.0))])
def test_fp8_kv_cache_kernels(gpu, D, scales):
    """FP8 e4m3fn KV pages: the RoPE/KV-write kernel stores exactly the reference's rounded
    bytes (k / k_scale, v / v_scale, saturated), and decode + prefill attention over those
    pages match the fp32 reference reading the same bytes."""
    torch.manual_seed(21)
    Hkv, G = 2, 4
    Hq = Hkv * G
    ctxs, qls = [700, 64, 130], [300, 64, 1]
    nb = sum((c + 63) // 64 for c in ctxs) + 2
    kc = torch.zeros(nb, Hkv, 64, D, dtype=torch.uint8, device=gpu).view(torch.float8_e4m3fn)
    vc = torch.zeros(nb, Hkv, D, 64, dtype=torch.uint8, device=gpu).view(torch.float8_e4m3fn)
    kc_r, vc_r = kc.cpu().clone(), vc.cpu().clone()
    # write every context position through the kernel (tiled path: T >= 64; per-token: T < 64)
    perm = torch.randperm(nb).tolist()
    bt = torch.zeros(len(ctxs), max((c + 63) // 64 for c in ctxs), dtype=torch.int32)
    k = 0
    for i, c in enumerate(ctxs):
        for j in range((c + 63) // 64):
            bt[i, j] = perm[k]
            k += 1
    cs = ops.rope_cos_sin(4096, D).to(gpu)
    for i, c in enumerate(ctxs):
        for lo, hi in ((0, c - 7), (c - 7, c)):
            T = hi - lo
            qkv = _bf(T, (Hq + 2 * Hkv) * D, dev=gpu, scale=4.0)
            pos = torch.arange(lo, hi, dtype=torch.int32, device=gpu)
            slots = (bt[i, pos.cpu().long() // 64] * 64 + pos.cpu() % 64).to(torch.int32).to(gpu)
            q_r = qkv.cpu().clone()
            ops.rope_cache_(qkv, pos, cs, slots, kc, vc, Hq, Hkv, D, kv_scales=scales)
            ref.rope_cache_(q_r, pos.cpu(), cs.cpu(), slots.cpu(), kc_r, vc_r, Hq, Hkv, D, kv_scales=scales)
    for got, want in ((kc, kc_r), (vc, vc_r)):
        diff = (got.cpu().view(torch.uint8).int() - want.view(torch.uint8).int()).abs()
        assert (diff > 1).sum() == 0 and (diff == 1).float().mean() < 1e-3   # RNE ties aside
    bt = bt.to(gpu)
    kc_r, vc_r = kc.cpu(), vc.cpu()   # the reference reads the kernel's bytes
    scale = 1 / math.sqrt(D)
    q = _bf(len(ctxs), Hq * D, dev=gpu)
    ctx = torch.tensor(ctxs, dtype=torch.int32, device=gpu)
    ws = ops.DecodeWorkspace(len(ctxs), Hq, Hkv, max(ctxs), gpu, D=D)
    out = ops.decode_attention(q, kc, vc, bt, ctx, Hq, Hkv, max(ctxs), scale, ws=ws, kv_scales=scales)
    o_ref = ref.decode_attention(q.cpu().float(), kc_r, vc_r, bt.cpu(), ctx.cpu(), Hq, Hkv, scale, D=D, kv_scales=scales)
    _close_rows(out, o_ref, width=D, rel=2e-2, peak=3e-2)
    cu = torch.tensor([0] + list(torch.tensor(qls).cumsum(0).tolist()), dtype=torch.int32, device=gpu)
    qp = _bf(sum(qls), Hq * D, dev=gpu)
    out = ops.prefill_attention_paged(qp, kc, vc, bt, cu, ctx, Hq, Hkv, D, max(qls), scale, kv_scales=scales)
    o_ref = ref.prefill_attention_paged(qp.cpu().float(), kc_r, vc_r, bt.cpu(), cu.cpu(), ctx.cpu(), Hq, Hkv, D, scale,
                                        kv_scales=scales)
    _close_rows(out, o_ref, width=D, rel=2e-2, peak=3e-2)


@pytest.mark.parametrize("D,H,causal", [(64, 16, False), (128, 8, True), (32, 12, False)])
def test_varlen_attention(gpu, D, H, causal):
    torch.manual_seed(4)
    lens = [5, 64, 130, 512, 1]
    cu = [0]
    for n in lens:
        cu.append(cu[-1] + n)
    T = cu[-1]
    qkv = _bf(T, 3 * H * D, dev=gpu)
    q, k, v = qkv[:, : H * D], qkv[:, H * D: 2 * H * D], qkv[:, 2 * H * D:]
    cu_t = torch.tensor(cu, dtype=torch.int32, device=gpu)
    scale = 1 / math.sqrt(D)
    out = ops.varlen_attention(q, k, v, cu_t, H, H, D, max(lens), scale, causal)
    o_ref = ref.varlen_attention(q.float(), k, v, cu_t, H, H, D, scale, causal)
    _close_rows(out, o_ref, width=D)


def test_sample(gpu):
    torch.manual_seed(5)
    B, V = 24, 128256
    logits = torch.randn(B, V, device=gpu) * 3
    temp = torch.tensor([0.0, 1.0, 0.7, 1.3] * 6, device=gpu)
    topk = torch.tensor([0, 0, 50, 1, 0, 10] * 4, dtype=torch.int32, device=gpu)
    topp = torch.tensor([1.0, 0.9, 1.0, 0.5, 0.7, 1.0] * 4, device=gpu)
    seeds = torch.arange(B, dtype=torch.int64, device=gpu) * 7919
    steps = torch.arange(B, dtype=torch.int64, device=gpu)
    lg_cpu = logits.cpu().clone()
    tok, lp = ops.sample(logits.clone(), temp, topk, topp, seeds, steps)
    tok_r, lp_r = ref.sample(lg_cpu, temp.cpu(), topk.cpu(), topp.cpu(), seeds.cpu(), steps.cpu())
    agree = (tok.cpu() == tok_r).float().mean().item()
    assert agree >= 0.9, f"only {agree:.2f} of draws agree with the reference"
    same = tok.cpu() == tok_r
    assert torch.allclose(lp.cpu()[same], lp_r[same], atol=1e-3)
    # every draw respects its own truncation
    for b in range(B):
        xs = lg_cpu[b] / (temp[b].item() if temp[b] > 0 else 1.0)
        t = int(tok[b])
        if int(topk[b]) > 0:
            assert xs[t] >= torch.topk(xs, int(topk[b])).values[-1]
        if temp[b] <= 0 or int(topk[b]) == 1:
            assert t == int(torch.argmax(xs))


def test_sample_repetition_penalty(gpu):
    B, V = 2, 1000
    logits = torch.zeros(B, V, device=gpu)
    logits[:, 7] = 5.0
    logits[:, 9] = 4.0
    hist = torch.tensor([[7, -1], [3, 3]], dtype=torch.int32, device=gpu)
    pen = torch.tensor([2.0, 2.0], device=gpu)
    tok, _ = ops.sample(logits, torch.zeros(B, device=gpu), torch.zeros(B, dtype=torch.int32, device=gpu),
                        torch.ones(B, device=gpu), torch.zeros(B, dtype=torch.int64, device=gpu),
                        torch.zeros(B, dtype=torch.int64, device=gpu), pen, hist)
    assert tok.tolist() == [9, 7]


@pytest.mark.parametrize("nq,N,D", [(1, 5000, 1024), (37, 70000, 1024), (64, 12345, 384), (130, 4096, 256)])
def test_score_topk(gpu, nq, N, D):
    torch.manual_seed(6)
    Q = _bf(nq, D, dev=gpu)
    X = _bf(N, D, dev=gpu)
    bias = torch.randn(N, device=gpu)
    S = ops.score(Q, X, bias, 0.5)
    S_ref = ref.score(Q.cpu(), X.cpu(), bias.cpu(), 0.5)
    _close(S, S_ref, 2e-3, 1e-4)
    for k in (1, 4, 100):
        v, i = ops.topk(S, k)
        v_ref, _ = torch.topk(S.cpu(), k, dim=1)
        _close(v, v_ref, 0.0)
        # indices point at the reported scores
        assert torch.equal(torch.gather(S.cpu(), 1, i.cpu()), v.cpu())


def test_pool(gpu):
    torch.manual_seed(7)
    lens = [3, 1, 77]
    cu = torch.tensor([0, 3, 4, 81], dtype=torch.int32, device=gpu)
    h = _bf(81, 1024, dev=gpu)
    for mode in (0, 1):
        _close(ops.pool_l2norm(h, cu, mode, True), ref.pool_l2norm(h.cpu(), cu.cpu(), mode, True), 1e-4)
    X = _bf(1000, 1024, dev=gpu)
    _close(ops.row_sqnorm(X), ref.row_sqnorm(X.cpu()), 0.05, 1e-4)


def test_hard_negative_mining_gpu_matches_cpu(gpu):
    from nv_genai_amd.training.hard_negatives import mine_hard_negatives

    g = torch.Generator().manual_seed(0)
    q = torch.nn.functional.normalize(torch.randn(300, 128, generator=g), dim=1).bfloat16().float()
    p = torch.nn.functional.normalize(torch.randn(9000, 128, generator=g), dim=1).bfloat16().float()
    pos = [[i, (i * 13) % 9000] for i in range(300)]
    cpu = mine_hard_negatives(q, p, pos, margin=0.9, num_negs=8)
    gpu_ = mine_hard_negatives(q.cuda(), p.cuda(), pos, margin=0.9, num_negs=8, block=128)
    agree = sum(len(set(a) & set(b)) for a, b in zip(cpu, gpu_)) / sum(len(a) for a in cpu)
    assert agree > 0.97, agree


def test_dsp_fir_demod_resample_match_reference(gpu):
    """FM front-end kernels (K18) against the fp64 PyTorch reference."""
    from nv_genai_amd import ops
    from nv_genai_amd.dsp.design import decimator, firwin
    from nv_genai_amd.ops import reference as R

    g = torch.Generator().manual_seed(0)
    x = torch.complex(torch.randn(5888, generator=g), torch.randn(5888, generator=g))
    taps = torch.tensor(firwin(101, 100e3, 1e6), dtype=torch.float32)
    hist = torch.complex(torch.randn(100, generator=g), torch.randn(100, generator=g))
    for h in (None, hist):
        got = ops.fir_c64(x.cuda(), taps.cuda(), None if h is None else h.cuda()).cpu()
        ref = R.fir_c64(x, taps, h)
        assert (got - ref).abs().max() < 1e-4
    lp = R.fir_c64(x, taps)
    for prev in (None, 0.3 - 0.2j):
        got = ops.fm_demod(lp.cuda(), prev).cpu()
        assert (got - R.fm_demod(lp, prev)).abs().max() < 1e-5
    d = decimator(62)
    dm = R.fm_demod(lp)
    h = torch.from_numpy(d.taps)
    yf, yi = ops.resample_pcm(dm.cuda(), h.cuda(), d.down, d.pre, d.n_out(dm.numel()), 10.0)
    rf, ri = R.resample_pcm(dm, h, d.down, d.pre, d.n_out(dm.numel()), 10.0)
    assert (yf.cpu() - rf).abs().max() < 1e-4
    assert (yi.cpu().int() - ri.int()).abs().max() <= 1


def test_sdr_pipeline_gpu_recovers_tone(gpu):
    import numpy as np

    from nv_genai_amd.dsp.replay import fm_modulate
    from nv_genai_amd.dsp.sdr import SDRPipeline

    fs_a = 16000
    t = np.arange(fs_a) / fs_a
    audio = 0.5 * np.sin(2 * np.pi * 440 * t).astype(np.float32)
    iq, _ = fm_modulate(audio, fs_a, 1e6, deviation=20_000)
    p = SDRPipeline(device="cuda", stateful=True)
    outs = [p.process(torch.from_numpy(iq[i:i + 5888]))[0].cpu() for i in range(0, len(iq), 5888)]
    y = torch.cat(outs).numpy()[200:]
    spec = np.abs(np.fft.rfft(y))
    f = np.fft.rfftfreq(len(y), 1 / (1e6 / 62))
    assert abs(f[spec.argmax()] - 440) < 5


def test_sample_odd_vocab_and_masked_logits(gpu):
    """Scalar-tail path (V % 4 != 0) and -inf (masked) logits in the fused max/partition pass."""
    torch.manual_seed(9)
    B, V = 6, 1001
    logits = torch.randn(B, V, device=gpu) * 2
    logits[:, ::3] = float("-inf")
    temp = torch.tensor([0.0, 0.8, 0.8, 1.0, 0.5, 0.0], device=gpu)
    topk = torch.tensor([0, 0, 20, 0, 5, 1], dtype=torch.int32, device=gpu)
    topp = torch.tensor([1.0, 0.9, 1.0, 0.6, 1.0, 1.0], device=gpu)
    seeds = torch.arange(B, dtype=torch.int64, device=gpu)
    steps = torch.zeros(B, dtype=torch.int64, device=gpu)
    tok, lp = ops.sample(logits.clone(), temp, topk, topp, seeds, steps)
    tok_r, lp_r = ref.sample(logits.cpu(), temp.cpu(), topk.cpu(), topp.cpu(), seeds.cpu(), steps.cpu())
    assert (tok.cpu() % 3 != 0).all()
    assert tok.cpu()[0] == tok_r[0] and torch.isfinite(lp).all()
    assert (tok.cpu() == tok_r).float().mean() >= 0.8


def _kept_set(xs, k, p, slack):
    """Reference truncation in float64: top-k, then the top-p nucleus widened by `slack`."""
    xs = xs.double()
    keep = torch.ones_like(xs, dtype=torch.bool)
    if 0 < k < xs.numel():
        keep &= xs >= torch.topk(xs, k).values[-1]
    if p < 1.0:
        pm = torch.exp(xs - xs.max()) * keep
        order = torch.argsort(xs, descending=True)
        cs = torch.cumsum(pm[order], 0)
        cut = int(torch.searchsorted(cs, torch.tensor([min(p + slack, 1.0) * float(pm.sum())], dtype=cs.dtype)))
        keep &= xs >= xs[order[min(cut, xs.numel() - 1)]]
    return keep


def test_sample_threshold_fast_path_and_fallbacks(gpu):
    """Rows chosen to take each threshold route of sampling.hip: the binned fast path (peaky and
    flat rows), the radix fallback for a crossing in the far tail (p close to 1), for a crossing
    bin with more than 2048 keys (quantised logits, a constant row), and top-k followed by top-p.
    Every draw must lie in the reference's kept set, and most draws equal the reference's."""
    torch.manual_seed(21)
    V = 128256
    rows = [
        (torch.randn(V) * 3, 0.2, 0, 0.7),                   # peaky, fast
        (torch.randn(V) * 0.5, 1.0, 0, 0.95),                # flat, fast
        (torch.randn(V) * 0.5, 1.0, 0, 0.9999),              # crossing in the tail: radix
        (torch.round(torch.randn(V) * 4) / 2, 1.0, 0, 0.5),  # thousands of ties per bin: radix
        (torch.zeros(V), 1.0, 0, 0.5),                       # constant row: keep everything
        (torch.randn(V) * 3, 1.0, 50, 1.0),                  # top-k fast
        (torch.round(torch.randn(V) * 4) / 2, 1.0, 3000, 1.0),  # top-k over a tie bin: radix
        (torch.randn(V) * 2, 0.8, 200, 0.8),                 # top-k then top-p
        (torch.randn(V) * 2, 0.05, 0, 0.9),                  # near-greedy temperature
    ]
    B = len(rows)
    logits = torch.stack([r[0] for r in rows]).float()
    temp = torch.tensor([r[1] for r in rows])
    topk = torch.tensor([r[2] for r in rows], dtype=torch.int32)
    topp = torch.tensor([r[3] for r in rows])
    seeds = torch.arange(B, dtype=torch.int64) * 131 + 7
    steps = torch.arange(B, dtype=torch.int64)
    agree = 0
    for rep in range(4):
        st = steps + rep * 17
        tok, lp = ops.sample(logits.to(gpu), temp.to(gpu), topk.to(gpu), topp.to(gpu), seeds.to(gpu), st.to(gpu))
        tok_r, lp_r = ref.sample(logits.clone(), temp, topk, topp, seeds, st)
        tok = tok.cpu()
        assert torch.isfinite(lp).all()
        agree += int((tok == tok_r).sum())
        for b in range(B):
            xs = logits[b] / temp[b]
            keep = _kept_set(xs, int(topk[b]), float(topp[b]), 1e-4)
            assert keep[int(tok[b])], f"row {b}: token {int(tok[b])} outside the kept set"
        same = tok == tok_r
        assert torch.allclose(lp.cpu()[same], lp_r[same], atol=1e-3)
    assert agree >= 0.9 * 4 * B, f"{agree} of {4 * B} draws agree with the reference"


def test_debug_sync_mode_checks_launches(gpu):
    """NGA_DEBUG_SYNC=1: every kernel binding checks its launch and synchronises its stream
    (fault localisation without a debugger); results are unchanged."""
    import os
    import subprocess
    import sys

    code = ("import torch; from nv_genai_amd import ops; from nv_genai_amd import _C;"
            "x = torch.randn(64, 4096, device='cuda').bfloat16(); w = torch.ones(4096, device='cuda').bfloat16();"
            "y = ops.rmsnorm(x, w, 1e-5); torch.cuda.synchronize();"
            "print(_C.debug_sync(), bool(torch.isfinite(y.float()).all()))")
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, NGA_DEBUG_SYNC="1"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().endswith("True True")


@pytest.mark.parametrize("mode,M,H", [(0, 37, 4096), (1, 19, 14336), (0, 16, 1024)])
def test_quant_fp8_rows(gpu, mode, M, H):
    """Row-wise e4m3fn quantiser (quant.hip) vs the fp32 reference: same scales, the same FP8
    codes except rare rounding ties, padded rows zero with scale 1."""
    torch.manual_seed(9)
    x = _bf(M, H * (2 if mode else 1), dev=gpu, scale=3.0)
    y, s = ops.quant_fp8_rows(x, mode)
    yr, sr = ref.quant_fp8_rows(x.cpu(), mode, y.shape[0])
    assert y.shape == yr.shape and y.dtype == torch.float8_e4m3fn
    _close(s, sr, 0.0, 1e-5)
    codes, codes_r = y.cpu().view(torch.uint8), yr.view(torch.uint8)
    assert (codes != codes_r).float().mean().item() < 1e-3
    deq = (y.float() * s)[:M].cpu()
    xv = x.float().cpu() if mode == 0 else torch.nn.functional.silu(x.float().cpu()[:, :H]) * x.float().cpu()[:, H:]
    assert float((deq - xv).norm() / xv.norm()) < 0.04


def test_fp8_linear_matches_dequantised_matmul(gpu):
    torch.manual_seed(10)
    x = _bf(50, 4096, dev=gpu)
    w = _bf(6144, 4096, dev=gpu, scale=0.02)
    x8, sx = ops.quant_fp8_rows(x)
    w8, sw = ops.quantize_weight_fp8(w)
    y = ops.fp8_linear(x8, sx, w8, sw, 50)
    y_ref = (x8.float() * sx)[:50] @ (w8.float() * sw.t()).t()
    _close(y, y_ref, 0.05, 0.01)
    exact = x.float() @ w.float().t()
    assert float((y.float() - exact).norm() / exact.norm()) < 0.06


@pytest.mark.parametrize("Hkv,G,window,ks,grid,impl", [(8, 4, 0, 1, 512, 2), (8, 4, 0, 2, 7, 2),
                                                       (2, 8, 0, 1, 13, 2), (4, 1, 0, 2, 64, 2),
                                                       (2, 4, 200, 1, 512, 2), (8, 4, 0, 1, 512, 1),
                                                       (2, 4, 200, 1, 9, 1)])
def test_prefill_attention_worklist(gpu, Hkv, G, window, ks, grid, impl):
    """Work-list mode of the 32x32 prefill kernel (the engine's mixed-step graphs): a step
    whose first rows are decode rows (left untouched) and whose prefill sequences are covered
    by the host-planned (sequence, row block) list, with a fixed grid smaller than the list
    (the persistent loop), against the fp32 reference."""
    D = 128
    Hq = Hkv * G
    nd = 5                                   # decode rows: one token each, not in the list
    ctxs = [300, 64, 1, 900, 33] + [1200, 700, 64, 1, 1500, 33]
    qls = [1] * nd + [940, 300, 64, 1, 1500, 1]
    kc, vc, bt = _paged_setup(ctxs, Hkv, D, gpu, seed=17)
    cu = [0]
    for ql in qls:
        cu.append(cu[-1] + ql)
    q = _bf(cu[-1], Hq * D, dev=gpu)
    cu_t = torch.tensor(cu, dtype=torch.int32, device=gpu)
    ctx_t = torch.tensor(ctxs, dtype=torch.int32, device=gpu)
    scale = 1 / math.sqrt(D)
    import numpy as np

    items = ops.plan_prefill_items(np.array(cu), np.array(ctxs), nd, len(ctxs), Hq, Hkv, window,
                                   rw=ops.worklist_rows(impl, Hq, Hkv))
    it_d = torch.zeros(len(items) + 9, 2, dtype=torch.int32, device=gpu)   # capacity > count
    it_d[: len(items)] = torch.from_numpy(items).to(gpu)
    n_d = torch.tensor([len(items)], dtype=torch.int32, device=gpu)
    out = torch.full((cu[-1], Hq * D), 7.0, dtype=torch.bfloat16, device=gpu)
    ops.prefill_attention_worklist(q, kc, vc, bt, cu_t, ctx_t, Hq, Hkv, scale, it_d, n_d, grid=grid, ks=ks,
                                   out=out, window=window, impl=impl)
    o_ref = ref.prefill_attention_paged(q[nd:].float(), kc, vc, bt[nd:], cu_t[nd:] - nd, ctx_t[nd:], Hq, Hkv, D,
                                        scale, True, window)
    _close_rows(out[nd:], o_ref, width=D)
    assert bool((out[:nd] == 7.0).all())     # decode rows untouched


def test_prefill_attention_worklist_fp8_and_d256(gpu):
    """The 16x16 kernel's work-list mode over fp8 e4m3fn pages (scales) and head_dim 256."""
    import numpy as np

    for D, fp8 in ((128, True), (256, False)):
        Hkv, G = 2, 4
        Hq = Hkv * G
        ctxs, qls = [9, 700, 130], [1, 300, 130]
        kc, vc, bt = _paged_setup(ctxs, Hkv, D, gpu, seed=23)
        scales = (2.0, 0.5) if fp8 else (1.0, 1.0)
        if fp8:
            kc, vc = (kc.float() / scales[0]).to(torch.float8_e4m3fn), (vc.float() / scales[1]).to(torch.float8_e4m3fn)
        cu = [0]
        for ql in qls:
            cu.append(cu[-1] + ql)
        q = _bf(cu[-1], Hq * D, dev=gpu)
        cu_t = torch.tensor(cu, dtype=torch.int32, device=gpu)
        ctx_t = torch.tensor(ctxs, dtype=torch.int32, device=gpu)
        items = ops.plan_prefill_items(np.array(cu), np.array(ctxs), 1, 3, Hq, Hkv, rw=64)
        it_d = torch.from_numpy(items).to(gpu)
        n_d = torch.tensor([len(items)], dtype=torch.int32, device=gpu)
        out = torch.zeros(cu[-1], Hq * D, dtype=torch.bfloat16, device=gpu)
        ops.prefill_attention_worklist(q, kc, vc, bt, cu_t, ctx_t, Hq, Hkv, D ** -0.5, it_d, n_d, grid=33,
                                       out=out, impl=1, kv_scales=scales)
        o_ref = ref.prefill_attention_paged(q[1:].float().cpu(), kc.cpu(), vc.cpu(), bt[1:].cpu(), cu_t[1:].cpu() - 1,
                                            ctx_t[1:].cpu(), Hq, Hkv, D, D ** -0.5, kv_scales=scales)
        _close_rows(out[1:], o_ref, width=D, rel=2e-2 if fp8 else 1e-2, peak=3e-2)


@pytest.mark.parametrize("dma", ["1", "2"])
def test_decode_attention_skip_empty_rows(gpu, dma, kernel_form, monkeypatch):
    """skip_empty: rows with ctx 0 are not written (the mixed-step graph's decode launch
    covers a bucket of rows whose tail belongs to the prefill tokens)."""
    kernel_form("decode_dma", dma)
    Hkv, G, D = 8, 4, 128
    Hq = Hkv * G
    ctxs = [100, 0, 700, 0]
    kc, vc, bt = _paged_setup([max(c, 1) for c in ctxs], Hkv, D, gpu)
    ctx = torch.tensor(ctxs, dtype=torch.int32, device=gpu)
    q = _bf(4, Hq * D, dev=gpu)
    for ppp in (None, 1):
        ws = ops.DecodeWorkspace(4, Hq, Hkv, 700, gpu, ppp)
        out = torch.full((4, Hq * D), 3.0, dtype=torch.bfloat16, device=gpu)
        ops.decode_attention(q, kc, vc, bt, ctx, Hq, Hkv, 700, 1 / math.sqrt(D), out=out, ws=ws, skip_empty=True)
        assert bool((out[1] == 3.0).all()) and bool((out[3] == 3.0).all())
        o_ref = ref.decode_attention(q.float(), kc, vc, bt, ctx, Hq, Hkv, 1 / math.sqrt(D))
        _close_rows(out[[0, 2]], o_ref[[0, 2]], width=D)


def test_embedding_gather(gpu):
    """embedding.hip: rows of the local vocabulary shard, zeros outside it, bf16 scale."""
    torch.manual_seed(12)
    table = _bf(1000, 4096, dev=gpu)
    ids = torch.tensor([0, 999, 5, 1000, 1500, 2999, 2000, 7], dtype=torch.int32, device=gpu)
    for lo, scale in ((0, 1.0), (1000, 1.0), (2000, 64.0)):
        got = ops.embedding(ids, table, lo, scale)
        want = ref.embedding(ids.cpu(), table.cpu(), lo, scale)
        assert torch.equal(got.cpu(), want)


# ------------------------------------------------------------ decode-shape projection GEMM
def _skinny_ref(x, w, epi):
    y = x.float().cpu() @ w.float().cpu().t()
    if epi == 2:
        F = w.shape[0] // 2
        y = torch.nn.functional.silu(y[:, :F]) * y[:, F:]
    return y


@pytest.mark.parametrize("M", [1, 17, 64, 200, 256, 512])
def test_skinny_gemm_every_cfg(gpu, M):
    """Every tile configuration x epilogue (bf16, fp32 K-split slabs, fused SwiGLU) against the
    fp32 reference, including ragged token tiles (M = 1, 17, 200) and a ragged last weight
    block (N = 1000 with BN 64-256); per-row relative error."""
    C = ops.kernels()
    torch.manual_seed(M)
    K = 1024
    x = _bf(M, K, dev=gpu)
    w = _bf(1000, K, dev=gpu, scale=0.05)
    wg = _bf(2 * 512, K, dev=gpu, scale=0.05)
    ref0, ref2 = _skinny_ref(x, w, 0), _skinny_ref(x, wg, 2)
    # SwiGLU for tiles whose BN / 2 does not divide 512 (BN 224: 112 features per block)
    wg7 = _bf(2 * 448, K, dev=gpu, scale=0.05)
    ref7 = _skinny_ref(x, wg7, 2)
    for cfg in range(C.skinny_cfg_count()):
        BN, BM = C.skinny_cfg(cfg)[:2]
        BK = C.skinny_cfg(cfg)[5]     # 64, or 32 (64-B LDS rows, twice the stages per KiB)
        _close_rows(ops.skinny_gemm(x, w, cfg, 1, 0), ref0, rel=1e-2)
        for s in (2, 5):
            P = ops.skinny_gemm(x, w, cfg, s, 1)
            _close_rows(P.sum(0), ref0, rel=1e-4)
            _close_rows(ops.splitk_reduce(P), ref0, rel=1e-2)
        F, wgc, refc = (512, wg, ref2) if 512 % (BN // 2) == 0 else (448, wg7, ref7)
        if F % (BN // 2) == 0:
            y2 = ops.skinny_gemm(x, wgc, cfg, 1, 2)
            _close_rows(y2, refc, rel=2e-2)
            # tile-packed weights and the rotated K walk: the same products (fp32 sums in
            # another order for krot)
            if BK == 64:
                assert torch.equal(ops.skinny_gemm(x, ops.pack_weight(wgc, BN, 2), cfg, 1, 2, n_out=F), y2)
        if BK != 64:   # packed operands are 64-deep tiles: refused for BK 32 tiles
            with pytest.raises(RuntimeError, match="packed operands"):
                ops.skinny_gemm(x, ops.pack_weight(w, BN), cfg, 1, 0, n_out=1000)
            _close_rows(ops.skinny_gemm(x, w, cfg, 3, 1, krot=1).sum(0), ref0, rel=1e-4)
            continue
        y0 = ops.skinny_gemm(x, w, cfg, 1, 0)
        assert torch.equal(ops.skinny_gemm(x, ops.pack_weight(w, BN), cfg, 1, 0, n_out=1000), y0)
        assert torch.equal(ops.skinny_gemm(ops.pack_rows(x, BM), ops.pack_weight(w, BN), cfg, 1, 0, n_out=1000,
                                           x_rows=M, k_in=K), y0)
        _close_rows(ops.skinny_gemm(x, ops.pack_weight(w, BN), cfg, 3, 1, n_out=1000, krot=1).sum(0), ref0,
                    rel=1e-4)


@pytest.mark.parametrize("M", [1, 2, 3, 4])
@pytest.mark.parametrize("N,K", [(37, 1000), (4096, 4096), (300, 14336)])
def test_gemv(gpu, M, N, K):
    """Weight-streaming GEMV (M <= 4) in its three epilogues against fp32: a ragged last wave
    (N % 4), a K that is not a multiple of the 512-element step, and the down projection's K."""
    torch.manual_seed(M + N)
    x = _bf(M, K, dev=gpu)
    w = _bf(2 * N, K, dev=gpu) * 0.05
    y_ref = x.cpu().float() @ w.cpu().float().t()
    _close_rows(ops.gemv(x, w[:N].contiguous(), 0), y_ref[:, :N], rel=1e-2)
    y1 = ops.gemv(x, w[:N].contiguous(), 1)
    assert y1.dtype == torch.float32
    _close_rows(y1, y_ref[:, :N], rel=1e-4)
    sw = torch.nn.functional.silu(y_ref[:, :N]) * y_ref[:, N:]
    _close_rows(ops.gemv(x, w, 2), sw, rel=1e-2)


def test_splitk_swiglu(gpu):
    """silu(sum of gate slabs) * sum of up slabs, against fp32."""
    torch.manual_seed(4)
    S, M, F = 3, 45, 1024
    P = torch.randn(S, M, 2 * F, device=gpu)
    s_ = P.cpu().sum(0)
    y_ref = torch.nn.functional.silu(s_[:, :F]) * s_[:, F:]
    y = ops.splitk_swiglu(P)
    _close_rows(y, y_ref, rel=1e-2)


def test_splitk_add_rmsnorm(gpu):
    torch.manual_seed(3)
    S, M, H = 4, 77, 4096
    P = torch.randn(S, M, H, device=gpu) * 0.3
    resid, w = _bf(M, H, dev=gpu), _bf(H, dev=gpu)
    r_ref = resid.cpu().float() + P.cpu().sum(0)
    y_ref = ref.rmsnorm(r_ref.to(torch.bfloat16).float(), w.cpu().float(), 1e-5)
    y = ops.splitk_add_rmsnorm(resid, P, w, 1e-5)
    _close_rows(resid, r_ref, rel=5e-3)
    _close_rows(y, y_ref, rel=1e-2)


def _table_cases():
    """(N, K, shape, M, cfg, split) of every kernel entry of the shipped decode-shape table."""
    import json

    from nv_genai_amd.ops.skinny import ASSET

    with open(ASSET) as f:
        doc = json.load(f)
    out = []
    for key, ent in doc["table"].items():
        n, k = (int(v) for v in key.split("x"))
        for m, c in sorted(ent["by_m"].items(), key=lambda kv: int(kv[0])):
            if c != "lib":
                out.append((n, k, ent["shape"], int(m), int(c[0]), int(c[1])))
    return out


def test_skinny_table_production_shapes(gpu):
    """Every (cfg, split) the shipped table (assets/skinny_gemm_gfx950.json) picks — llama3-8b,
    llama3-70b at TP=8 (rank shards) and TP=1 — at its own M and real shape, run the way the
    model runs it WITH its consumer, against fp32: q/k/v K-split slabs summed by the RoPE /
    KV-write kernel (q, k, v and both caches), o / down slabs summed by the residual add +
    RMSNorm kernel, gate / up through the SwiGLU epilogue (split 1) or the split-K SwiGLU
    kernel, the LM head's fp32 logits. Per-row relative error."""
    cases = _table_cases()
    assert len(cases) > 100
    by_shape = {}
    for c in cases:
        by_shape.setdefault((c[0], c[1], c[2]), []).append(c[3:])
    eps, D = 1e-5, 128
    for (N, K, shape), rows in by_shape.items():
        torch.manual_seed(N + K)
        w = _bf(N, K, dev=gpu, scale=0.02)
        for M, cfg, split in rows:
            x = _bf(M, K, dev=gpu)
            ref = x.float() @ w.float().t()
            tag = f"{shape} {N}x{K} M={M} cfg={cfg} split={split}"
            if shape == "qkv":
                Hkv = N // D // 10 if N // D % 10 == 0 else N // D // 6    # 8B: 32+8+8, 70B: 64+8+8 / 8+1+1
                Hq = N // D - 2 * Hkv
                P = ops.skinny_gemm(x, w, cfg, split, 1 if split > 1 else 0)
                pos = torch.randint(0, 4000, (M,), dtype=torch.int32, device=gpu)
                cs = ops.rope_cos_sin(4096, D).to(gpu)
                nb = (M + 63) // 64 + 2
                kc, vc = _make_cache(nb, Hkv, D, gpu)
                slots = torch.randperm(nb * 64, device=gpu)[:M].to(torch.int32)
                kc2, vc2 = kc.clone(), vc.clone()
                want = ref.to(torch.bfloat16)
                ops.rope_cache_(want, pos, cs, slots, kc, vc, Hq, Hkv, D)
                if split > 1:
                    got = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
                    ops.rope_cache_(got, pos, cs, slots, kc2, vc2, Hq, Hkv, D, partial=ops.PartialSum(P))
                else:
                    got = P
                    ops.rope_cache_(got, pos, cs, slots, kc2, vc2, Hq, Hkv, D)
                _close_rows(got, want, width=D, rel=2e-2)
                _close_rows(kc2.float(), kc.float(), width=D, rel=2e-2)
                _close_rows(vc2.float().transpose(-1, -2), vc.float().transpose(-1, -2), width=D, rel=2e-2)
            elif shape in ("o", "down"):
                resid = _bf(M, N, dev=gpu)
                nw = (1.0 + 0.1 * torch.randn(N, device=gpu)).to(torch.bfloat16)
                r32 = resid.float() + ref
                want = r32 * torch.rsqrt(r32.pow(2).mean(1, keepdim=True) + eps) * nw.float()
                P = ops.skinny_gemm(x, w, cfg, split, 1)
                out = ops.splitk_add_rmsnorm(resid, P, nw, eps)
                _close_rows(resid, r32, rel=1e-2)
                _close_rows(out, want, rel=2e-2)
                _close_rows(P.sum(0), ref, rel=1e-4)
            elif shape == "gate_up":
                F = N // 2
                want = torch.nn.functional.silu(ref[:, :F]) * ref[:, F:]
                got = (ops.skinny_gemm(x, w, cfg, 1, 2) if split == 1
                       else ops.splitk_swiglu(ops.skinny_gemm(x, w, cfg, split, 1)))
                _close_rows(got, want, rel=2e-2)
            else:   # lm_head: fp32 logits straight from the accumulators
                got = ops.skinny_gemm(x, w, cfg, split, 1)
                _close_rows(got.sum(0), ref, rel=1e-4)
            del ref
        del w
        torch.cuda.empty_cache()


def test_packed_upload_scatters_segments(gpu):
    """ops/staging.PackedUpload: the used rows of several pinned buffers (int32, fp32, int64,
    2-D rows, a ragged word count) reach their device buffers through one scatter kernel that
    reads the mapped host staging in place, rows past `rows` untouched; both staging halves in
    turn; oversize rows refused. Then three uploads queued behind a busy stream, the sources
    rewritten after each: the third reuses the first's staging half only after the first
    kernel has read it."""
    from nv_genai_amd.ops.staging import PackedUpload

    g = torch.Generator().manual_seed(3)
    specs = [((1000,), torch.int32), ((77,), torch.float32), ((300,), torch.int64), ((40, 37), torch.int32),
             ((5,), torch.float32)]
    hs = [torch.randint(-1000, 1000, s, generator=g).to(dt).pin_memory() for s, dt in specs]
    ds = [torch.full(s, -7, dtype=dt, device=gpu) for s, dt in specs]
    up = PackedUpload(gpu, sum(h.numel() * h.element_size() + 16 for h in hs))
    for it, rows in enumerate(([999, 77, 1, 13, 5], [3, 0, 300, 40, 2])):
        for h in hs:
            h.copy_(torch.randint(-1000, 1000, h.shape, generator=g).to(h.dtype))
        before = [d.clone() for d in ds]
        up.upload(list(zip(hs, ds, rows)))
        torch.cuda.synchronize()
        for h, d, b, r in zip(hs, ds, before, rows):
            assert torch.equal(d[:r].cpu(), h[:r]), (it, r)
            assert torch.equal(d[r:], b[r:])
    assert up.uploads == 2
    with pytest.raises(ValueError):
        up.upload([(hs[0], ds[0], 1001)])
    want = []
    torch.cuda._sleep(20_000_000)
    for i in range(3):
        for h in hs:
            h.copy_(torch.randint(-1000, 1000, h.shape, generator=g).to(h.dtype))
        want.append(hs[i][:5].clone())
        up.upload([(hs[i], ds[i], 5)])
    torch.cuda.synchronize()
    for i in range(3):
        assert torch.equal(ds[i][:5].cpu(), want[i]), i
