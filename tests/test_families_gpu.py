"""GPU numerics of the kernels behind the non-Llama decoder families (Mistral / StarCoder2
sliding window, Gemma head_dim 256 + GeGLU, StarCoder2 LayerNorm + tanh GELU, Mixtral MoE
grouped GEMMs), each against the fp32 PyTorch reference of the same op, plus an end-to-end
prefill-logit check of a small model of every family on the HIP path vs the CPU reference."""
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


def test_add_layernorm_geglu_gelu_tanh(gpu):
    torch.manual_seed(0)
    for H in (1024, 4608, 6144):
        r, d, g, b = _bf(29, H, dev=gpu), _bf(29, H, dev=gpu), _bf(H, dev=gpu), _bf(H, dev=gpu)
        r_ref = r.cpu().clone()
        y = ops.add_layernorm(r, d, g, b, 1e-5)
        y_ref = ref.add_layernorm(r_ref, d.cpu(), g.cpu(), b.cpu(), 1e-5)
        _close(r, r_ref, 0.02, 0.01)
        _close(y, y_ref, 0.06, 0.01)
    gu = _bf(23, 2 * 24576, dev=gpu)
    _close(ops.gelu_tanh_mul(gu), ref.gelu_tanh_mul(gu.cpu()), 0.05, 0.01)
    h, bias = _bf(17, 12288, dev=gpu), _bf(12288, dev=gpu)
    h_ref = h.cpu().clone()
    ops.bias_gelu_(h, bias, approximate=True)
    ref.bias_gelu_(h_ref, bias.cpu(), approximate=True)
    _close(h, h_ref, 0.03, 0.01)


@pytest.mark.parametrize("T", [7, 130])
def test_rope_cache_head_dim_256(gpu, T):
    torch.manual_seed(2)
    Hq, Hkv, D = 8, 1, 256
    qkv = _bf(T, (Hq + 2 * Hkv) * D, dev=gpu)
    pos = torch.randint(0, 4000, (T,), dtype=torch.int32, device=gpu)
    cs = ops.rope_cos_sin(4096, D, 10000.0).to(gpu)
    nb = (T + 63) // 64 + 3
    kc, vc = _bf(nb, Hkv, 64, D, dev=gpu), _bf(nb, Hkv, D, 64, dev=gpu)
    slots = torch.randperm(nb * 64, device=gpu)[:T].to(torch.int32)
    slots[3] = -1
    qkv_r, kc_r, vc_r = qkv.cpu().clone(), kc.cpu().clone(), vc.cpu().clone()
    ops.rope_cache_(qkv, pos, cs, slots, kc, vc, Hq, Hkv, D)
    ref.rope_cache_(qkv_r, pos.cpu(), cs.cpu(), slots.cpu(), kc_r, vc_r, Hq, Hkv, D)
    _close(qkv, qkv_r, 0.03, 0.01)
    _close(kc, kc_r, 0.03, 0.01)
    _close(vc, vc_r, 1e-6)


def _paged(ctxs, Hkv, D, dev, seed=0):
    torch.manual_seed(seed)
    pages = [(c + 63) // 64 for c in ctxs]
    nb = sum(pages) + 2
    kc, vc = _bf(nb, Hkv, 64, D, dev=dev), _bf(nb, Hkv, D, 64, dev=dev)
    perm = torch.randperm(nb).tolist()
    bt = torch.zeros(len(ctxs), max(pages), dtype=torch.int32)
    k = 0
    for i, p in enumerate(pages):
        for j in range(p):
            bt[i, j] = perm[k]
            k += 1
    return kc, vc, bt.to(dev)


@pytest.mark.parametrize("D,G,window,ppp", [(256, 8, 0, None), (256, 1, 0, 2), (128, 4, 200, None),
                                            (128, 4, 200, 1), (256, 8, 300, None), (128, 8, 64, None)])
@pytest.mark.parametrize("dma", ["1", "2"])
def test_decode_attention_dim_and_window(gpu, D, G, window, ppp, dma, kernel_form, monkeypatch):
    kernel_form("decode_dma", dma)   # head_dim 128 pages: whole-page / ring DMA kernel
    Hkv = 2 if G < 8 else 1
    Hq = Hkv * G
    ctxs = [1, 63, 64, 65, 199, 200, 201, 700, 1333]
    kc, vc, bt = _paged(ctxs, Hkv, D, gpu)
    B = len(ctxs)
    q = _bf(B, Hq * D, dev=gpu)
    ctx = torch.tensor(ctxs, dtype=torch.int32, device=gpu)
    scale = 1 / math.sqrt(D)
    ws = ops.DecodeWorkspace(B, Hq, Hkv, max(ctxs), gpu, ppp, D=D)
    out = ops.decode_attention(q, kc, vc, bt, ctx, Hq, Hkv, max(ctxs), scale, ws=ws, window=window)
    o_ref = ref.decode_attention(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), ctx.cpu(), Hq, Hkv, scale,
                                 D=D, window=window)
    _close(out, o_ref, 0.02)


@pytest.mark.parametrize("D,window", [(256, 0), (128, 100), (256, 150), (64, 70)])
def test_prefill_attention_dim_and_window(gpu, D, window):
    Hkv, G = 2, 4
    Hq = Hkv * G
    ctxs = [100, 700, 64, 1, 515]
    qls = [100, 300, 64, 1, 129]
    kc, vc, bt = _paged(ctxs, Hkv, D, gpu, seed=3)
    cu = [0]
    for ql in qls:
        cu.append(cu[-1] + ql)
    q = _bf(cu[-1], Hq * D, dev=gpu)
    cu_t = torch.tensor(cu, dtype=torch.int32, device=gpu)
    ctx = torch.tensor(ctxs, dtype=torch.int32, device=gpu)
    scale = 1 / math.sqrt(D)
    out = ops.prefill_attention_paged(q, kc, vc, bt, cu_t, ctx, Hq, Hkv, D, max(qls), scale,
                                      window=window)
    o_ref = ref.prefill_attention_paged(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), cu_t.cpu(), ctx.cpu(),
                                        Hq, Hkv, D, scale, window=window)
    _close(out, o_ref, 0.02)


@pytest.mark.parametrize("T,E,k,act", [(5, 8, 2, "silu"), (300, 8, 2, "silu"), (1200, 8, 2, "silu"),
                                       (77, 4, 1, "gelu_tanh"), (640, 16, 4, "silu")])
def test_moe_ffn_matches_reference(gpu, T, E, k, act):
    torch.manual_seed(T)
    H, F = 1024, 1792
    x = _bf(T, H, dev=gpu)
    router = _bf(E, H, dev=gpu)
    w13 = _bf(E, 2 * F, H, dev=gpu, scale=0.03)
    w2 = _bf(E, H, F, dev=gpu, scale=0.03)
    y = ops.moe_ffn(x, router, w13, w2, k, act=act)
    y_ref = ref.moe_ffn(x.cpu(), router.cpu(), w13.cpu(), w2.cpu(), k, act=act)
    _close(y, y_ref, 0.02, 0.02)
    # expert parallel: two halves of the experts sum to the whole layer
    h = E // 2
    y0 = ops.moe_ffn(x, router, w13[:h].contiguous(), w2[:h].contiguous(), k, expert0=0, act=act)
    y1 = ops.moe_ffn(x, router, w13[h:].contiguous(), w2[h:].contiguous(), k, expert0=h, act=act)
    _close(y0.float() + y1.float(), y_ref, 0.03, 0.02)


def test_moe_ffn_graph_capture(gpu):
    """The MoE path (route, align, grouped GEMMs, combine) replays inside a hipGraph."""
    torch.manual_seed(9)
    T, H, F, E, k = 64, 1024, 1792, 8, 2
    x = _bf(T, H, dev=gpu)
    router = _bf(E, H, dev=gpu)
    w13 = _bf(E, 2 * F, H, dev=gpu, scale=0.03)
    w2 = _bf(E, H, F, dev=gpu, scale=0.03)
    ops.MoEWorkspace.get(T, k, E, gpu)
    eager = ops.moe_ffn(x, router, w13, w2, k)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.moe_ffn(x, router, w13, w2, k)
        with torch.cuda.graph(g, stream=s):
            out = ops.moe_ffn(x, router, w13, w2, k)
    torch.cuda.current_stream().wait_stream(s)
    x.copy_(_bf(T, H, dev=gpu))
    g.replay()
    torch.cuda.synchronize()
    _close(out, ref.moe_ffn(x.cpu(), router.cpu(), w13.cpu(), w2.cpu(), k), 0.02, 0.02)
    assert not torch.equal(out, eager)


@pytest.mark.parametrize("name", ["mistral-small", "mixtral-small", "gemma-small", "starcoder2-small"])
def test_family_engine_gpu_matches_cpu(gpu, name):
    """Prefill logits of the whole model on the HIP path vs the CPU reference path, then a few
    greedy hipGraph decode steps run and stay finite."""
    from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine, SamplingParams
    from nv_genai_amd.models.config import llama_config
    from nv_genai_amd.models.llama import LlamaModel
    from nv_genai_amd.parallel.dist import ParallelContext

    m = LlamaModel(llama_config(name), "cpu", pctx=ParallelContext(), seed=4)
    w = m.state_dict()
    cfg = dict(model=name, max_num_seqs=4, max_batched_tokens=2048, max_model_len=2048,
               kv_cache_blocks=64, graph_batch_sizes=(1, 2, 4))
    prompt = [(11 * i + 5) % 30000 + 10 for i in range(450)]
    logits = []
    for dev in ("cuda", "cpu"):
        eng = LLMEngine(EngineConfig(use_graphs=False, **cfg), device=dev, pctx=ParallelContext(), weights=w)
        eng.add_request(prompt, SamplingParams(temperature=0.0, max_tokens=1, ignore_eos=True))
        ids, pos, sl, cu, ctx, bt, sid, smp = eng._np
        kind, n, ntok = eng.sched.schedule(ids, pos, sl, cu, ctx, bt, sid, smp)
        cu_ = eng._np[3][: n + 1]
        eng._upload(n, ntok)
        logits.append(eng._prefill_forward(n, ntok, int((cu_[1:] - cu_[:-1]).max()),
                                           int(eng._np[4][:n].max())).float().cpu())
    lg, lc = logits
    rel = ((lg - lc).norm() / lc.norm()).item()
    assert rel < 0.03, f"{name}: relative logit error {rel:.4f}"
    eng = LLMEngine(EngineConfig(use_graphs=True, **cfg), device="cuda", pctx=ParallelContext(), weights=w)
    outs = eng.generate([prompt, prompt[:300]], SamplingParams(temperature=0.0, max_tokens=12, ignore_eos=True))
    assert all(len(r.output_ids) == 12 for r in outs)


def test_quick_gelu_kernel(gpu):
    torch.manual_seed(3)
    h, bias = _bf(33, 4096, dev=gpu), _bf(4096, dev=gpu)
    h_ref = h.cpu().clone()
    ops.bias_gelu_(h, bias, "quick")
    ref.bias_gelu_(h_ref, bias.cpu(), "quick")
    _close(h, h_ref, 0.03, 0.01)


def test_vision_tower_and_vlm_gpu(gpu):
    """CLIP ViT tower + projector on the HIP kernels vs the CPU reference path, then a VLM
    request (image features spliced into the prefill) through the GPU engine."""
    import io

    from PIL import Image

    from nv_genai_amd.engine.llm_engine import EngineConfig, SamplingParams
    from nv_genai_amd.models.vision import VisionLanguageModel, VisionTower, preprocess_image, vlm_config

    cfg = vlm_config("vlm-small")
    cpu_t = VisionTower(cfg.vision, "cpu", seed=3)
    g = torch.Generator().manual_seed(0)
    arr = (torch.rand(180, 240, 3, generator=g) * 255).to(torch.uint8).numpy()
    buf = io.BytesIO()
    Image.fromarray(arr).save(buf, format="PNG")
    img = buf.getvalue()
    pix = preprocess_image(img, cfg.vision).unsqueeze(0)
    want = cpu_t.forward(pix).float()
    gpu_t = VisionTower(cfg.vision, "cuda", weights=cpu_t.state_dict())   # same weights (the CPU
    # and GPU generators draw different random streams)
    got = gpu_t.forward(pix.to(gpu)).float().cpu()
    rel = ((got - want).norm() / want.norm()).item()
    assert rel < 0.03, rel
    vlm = VisionLanguageModel("vlm-small", device="cuda",
                              engine_cfg=EngineConfig(model="llama-small", max_num_seqs=4, max_batched_tokens=2048,
                                                      max_model_len=2048, kv_cache_blocks=64, graph_batch_sizes=(1, 2, 4)))
    msgs = [{"role": "user", "content": [{"type": "text", "text": "Describe this image in detail"},
                                          {"type": "image", "image": img}]}]
    r = vlm.generate([msgs, msgs], SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True))
    assert r[0].output_ids == r[1].output_ids and len(r[0].output_ids) == 8


def test_decoder_ranker_gpu_matches_cpu(gpu):
    """nv-rerank-qa-mistral-4b-layout reranker (bidirectional GQA varlen attention, head_dim
    128, mean pool + head) on the HIP kernels vs the CPU reference path."""
    from nv_genai_amd.engine.embed_engine import EmbeddingEngine

    q = "what does the quarterly report say about revenue?"
    ps = ["revenue grew twelve percent in the quarter", "the cafeteria menu changes weekly",
          "guidance for the next quarter was raised " * 20]
    from nv_genai_amd.models.ranker import DecoderRanker

    cpu_r = DecoderRanker("mistral-rerank-small", "cpu", seed=1)
    gpu_r = DecoderRanker("mistral-rerank-small", "cuda", weights=cpu_r.state_dict())
    g = torch.tensor(EmbeddingEngine("mistral-rerank-small", device="cuda", encoder=gpu_r).rerank(q, ps))
    c = torch.tensor(EmbeddingEngine("mistral-rerank-small", device="cpu", encoder=cpu_r).rerank(q, ps))
    assert torch.allclose(g, c, atol=0.03 * c.abs().max().item() + 1e-3), (g, c)


def test_sample_gemma_vocab_with_penalty(gpu):
    """256000-token rows (Gemma): penalty bitmap covers ids past 131072, sampling and greedy
    agree with the reference sampler."""
    B, V = 3, 256000
    torch.manual_seed(4)
    logits = torch.randn(B, V, device=gpu)
    logits[:, 200001] = 9.0
    logits[:, 150000] = 8.0
    hist = torch.tensor([[200001, -1], [5, 5], [150000, 200001]], dtype=torch.int32, device=gpu)
    pen = torch.tensor([2.0, 2.0, 3.0], device=gpu)
    zero_t = torch.zeros(B, device=gpu)
    tok, _ = ops.sample(logits.clone(), zero_t, torch.zeros(B, dtype=torch.int32, device=gpu), torch.ones(B, device=gpu),
                        torch.zeros(B, dtype=torch.int64, device=gpu), torch.zeros(B, dtype=torch.int64, device=gpu),
                        pen, hist)
    assert tok.tolist()[:2] == [150000, 200001]
    temp = torch.full((B,), 0.7, device=gpu)
    topk = torch.tensor([50, 0, 10], dtype=torch.int32, device=gpu)
    topp = torch.tensor([0.9, 0.7, 1.0], device=gpu)
    seeds = torch.arange(B, dtype=torch.int64, device=gpu)
    steps = torch.ones(B, dtype=torch.int64, device=gpu)
    t1, lp = ops.sample(logits.clone(), temp, topk, topp, seeds, steps)
    t2, _ = ref.sample(logits.cpu(), temp.cpu(), topk.cpu(), topp.cpu(), seeds.cpu(), steps.cpu())
    assert torch.isfinite(lp).all() and (t1.cpu() == t2).all()
