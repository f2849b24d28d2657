"""Decoder families beyond Llama: Mistral (sliding window),
Mixtral (sparse MoE), Gemma (GeGLU, head_dim 256, (1 + w) norms, scaled embedding) and
StarCoder2 (LayerNorm + biases, plain GELU MLP, sliding window).

Parity is pinned against the ``transformers`` implementations of the same architectures
(installed here; random weights of tiny configs, no checkpoint needed): our decoder loads the
HF state dict and must reproduce HF's logits for a prefill, and for a decode step against the
paged KV cache, on the CPU reference path (fp32 math on bf16 weights) — the same path the GPU
numerics tests compare the HIP kernels against."""
import pytest
import torch

from nv_genai_amd.models.config import llama_config
from nv_genai_amd.models.llama import AttnMeta, LlamaModel

transformers = pytest.importorskip("transformers")


def _hf(arch: str, cfg):
    rp = {"rope_theta": cfg.rope_theta, "rope_type": "default"}
    common = dict(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden, intermediate_size=cfg.ffn,
                  num_hidden_layers=cfg.layers, num_attention_heads=cfg.heads,
                  num_key_value_heads=cfg.kv_heads, max_position_embeddings=cfg.max_position,
                  rope_parameters=rp, bos_token_id=1, eos_token_id=2, pad_token_id=0,
                  attn_implementation="eager")
    if arch == "mistral":
        c = transformers.MistralConfig(head_dim=cfg.head_dim, sliding_window=cfg.sliding_window or None,
                                       rms_norm_eps=cfg.eps, **common)
        return transformers.MistralForCausalLM(c)
    if arch == "mixtral":
        c = transformers.MixtralConfig(head_dim=cfg.head_dim, num_local_experts=cfg.num_experts,
                                       num_experts_per_tok=cfg.experts_per_tok, rms_norm_eps=cfg.eps,
                                       sliding_window=None, **common)
        return transformers.MixtralForCausalLM(c)
    if arch == "gemma":
        c = transformers.GemmaConfig(head_dim=cfg.head_dim, hidden_act="gelu_pytorch_tanh",
                                     rms_norm_eps=cfg.eps, tie_word_embeddings=True, **common)
        return transformers.GemmaForCausalLM(c)
    if arch == "starcoder2":
        c = transformers.Starcoder2Config(sliding_window=cfg.sliding_window, norm_epsilon=cfg.eps,
                                          use_bias=True, hidden_act="gelu_pytorch_tanh",
                                          tie_word_embeddings=True, **common)
        return transformers.Starcoder2ForCausalLM(c)
    raise ValueError(arch)


def _perturb(m, arch):
    """Non-trivial norms and biases (HF initialises them to 1 / 0)."""
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "norm" in n and n.endswith("weight"):
                base = 0.0 if arch == "gemma" else 1.0
                p.copy_(base + 0.1 * torch.randn(p.shape, generator=g))
            elif n.endswith("bias"):
                p.copy_(0.02 * torch.randn(p.shape, generator=g))
            else:
                p.copy_(0.05 * torch.randn(p.shape, generator=g))


def _meta(T, ctx, kind, nblk=8):
    bt = torch.arange(nblk, dtype=torch.int32).unsqueeze(0)
    return AttnMeta(kind=kind, slots=torch.arange(ctx - T, ctx, dtype=torch.int32),
                    cu_q=torch.tensor([0, T], dtype=torch.int32),
                    ctx_lens=torch.tensor([ctx], dtype=torch.int32), block_tables=bt,
                    max_q_len=T, max_ctx=ctx)


@pytest.mark.parametrize("name", ["mistral-tiny", "mixtral-tiny", "gemma-tiny", "starcoder2-tiny"])
def test_family_matches_transformers(name):
    cfg = llama_config(name)
    torch.manual_seed(0)
    hf = _hf(cfg.arch, cfg).eval()
    _perturb(hf, cfg.arch)
    sd = {k: v.detach().clone() for k, v in hf.state_dict().items()}
    ours = LlamaModel(cfg, "cpu", dtype=torch.bfloat16, weights=sd)
    ours.allocate_kv_cache(8, 64)
    hf = hf.to(torch.bfloat16)

    T = 150 if cfg.sliding_window else 100      # longer than the tiny configs' 96-token window
    ids = torch.randint(3, cfg.vocab_size, (T + 1,), generator=torch.Generator().manual_seed(3))
    with torch.no_grad():
        ref = hf(ids.unsqueeze(0).long()).logits[0].float()        # [T+1, V]
        h = ours.forward(ids[:T].int(), torch.arange(T, dtype=torch.int32), _meta(T, T, "prefill"),
                         sample_idx=torch.tensor([T - 1]))
        lp = ours.logits(h)[0]
        h = ours.forward(ids[T:].int(), torch.tensor([T], dtype=torch.int32), _meta(1, T + 1, "decode"))
        ld = ours.logits(h)[0]
    for got, want in ((lp, ref[T - 1]), (ld, ref[T])):
        err = (got - want).abs().max().item() / want.abs().max().item()
        cos = torch.nn.functional.cosine_similarity(got, want, dim=0).item()
        assert cos > 0.999 and err < 0.05, (name, cos, err)
        assert got.argmax() == want.argmax()


def test_state_dict_round_trip_all_families():
    for name in ["mistral-tiny", "mixtral-tiny", "gemma-tiny", "starcoder2-tiny"]:
        cfg = llama_config(name)
        a = LlamaModel(cfg, "cpu", seed=5)
        b = LlamaModel(cfg, "cpu", weights=a.state_dict())
        for La, Lb in zip(a.layers, b.layers):
            assert La.keys() == Lb.keys()
            for k in La:
                assert torch.equal(La[k], Lb[k]), (name, k)
        assert torch.equal(a.final_norm, b.final_norm)
        assert (b.lm_head is b.embed) == cfg.tie_embeddings


def test_sliding_window_reference_semantics():
    """Key j is visible to query i iff i - W < j <= i, in prefill and decode alike."""
    from nv_genai_amd.ops import reference as ref

    torch.manual_seed(0)
    Hq, Hkv, D, W, ctx = 2, 1, 64, 40, 130
    kc = torch.randn(3, Hkv, 64, D, dtype=torch.bfloat16)
    vc = torch.randn(3, Hkv, D, 64, dtype=torch.bfloat16)
    bt = torch.tensor([[0, 1, 2]], dtype=torch.int32)
    q = torch.randn(ctx, Hq * D, dtype=torch.bfloat16)
    full = ref.prefill_attention_paged(q, kc, vc, bt, torch.tensor([0, ctx], dtype=torch.int32),
                                       torch.tensor([ctx], dtype=torch.int32), Hq, Hkv, D, 0.125,
                                       window=W)
    for i in (5, 39, 40, 41, 129):
        dec = ref.decode_attention(q[i:i + 1], kc, vc, bt, torch.tensor([i + 1], dtype=torch.int32),
                                   Hq, Hkv, 0.125, D=D, window=W)
        assert torch.allclose(dec[0].float(), full[i].float(), atol=1e-2), i


def test_moe_reference_matches_dense_expert_loop():
    from nv_genai_amd.ops import reference as ref

    torch.manual_seed(0)
    T, H, F, E, k = 9, 32, 48, 4, 2
    x = torch.randn(T, H, dtype=torch.bfloat16)
    router = torch.randn(E, H, dtype=torch.bfloat16)
    w13 = (0.1 * torch.randn(E, 2 * F, H)).to(torch.bfloat16)
    w2 = (0.1 * torch.randn(E, H, F)).to(torch.bfloat16)
    y = ref.moe_ffn(x, router, w13, w2, k).float()
    p = torch.softmax((x @ router.t()).float(), -1)
    want = torch.zeros(T, H)
    for t in range(T):
        w, ids = torch.topk(p[t], k)
        w = w / w.sum()
        for j in range(k):
            e = int(ids[j])
            gu = x[t].float() @ w13[e].float().t()
            h = (torch.nn.functional.silu(gu[:F]) * gu[F:]).to(torch.bfloat16).float()
            want[t] += w[j] * (h @ w2[e].float().t())
    assert torch.allclose(y, want, atol=2e-2, rtol=2e-2)
    # expert-parallel halves sum to the whole
    y0 = ref.moe_ffn(x, router, w13[:2], w2[:2], k, expert0=0).float()
    y1 = ref.moe_ffn(x, router, w13[2:], w2[2:], k, expert0=2).float()
    assert torch.allclose(y0 + y1, y, atol=2e-2)


def test_decoder_ranker_matches_dense_bidirectional_reference():
    """nv-rerank-qa-mistral-4b layout: decoder layers with a bidirectional mask, masked mean
    pool, linear head — our packed forward vs an explicit per-pair fp32 recomputation."""
    from nv_genai_amd.engine.embed_engine import EmbeddingEngine
    from nv_genai_amd.models.ranker import DecoderRanker
    from nv_genai_amd.training import functional as Fn

    eng = EmbeddingEngine("mistral-rerank-tiny", device="cpu")
    assert isinstance(eng.model, DecoderRanker)
    q = "which river flows through the capital?"
    ps = ["the capital sits on a wide river delta", "widgets are sold in boxes of twelve",
          "x " * 700]                                               # > 512 tokens: truncated END
    got = torch.tensor(eng.rerank(q, ps))
    m = eng.model.lm
    want = []
    for p in ps:
        ids = torch.tensor(eng.model.encode_pair(q, p))
        assert ids.numel() <= 512
        S = ids.numel()
        # bidirectional reference: the training forward with a full (non-causal) mask
        B = 1
        hq, hkv, D = m.hq, m.hkv, m.D
        cs = m.cos_sin[torch.arange(S)]
        cos, sin = cs[:, : D // 2].view(1, S, 1, -1), cs[:, D // 2:].view(1, S, 1, -1)
        x = torch.nn.functional.embedding(ids.unsqueeze(0), m.embed).float()
        for L in m.layers:
            h = Fn.rms_norm(x, L["attn_norm"], m.cfg.eps).float()
            qkv = h @ L["wqkv"].float().t()
            qq, kk, vv = qkv.split([hq * D, hkv * D, hkv * D], -1)
            qq = Fn.apply_rope(qq.view(B, S, hq, D), cos, sin).transpose(1, 2)
            kk = Fn.apply_rope(kk.view(B, S, hkv, D), cos, sin).transpose(1, 2)
            vv = vv.view(B, S, hkv, D).transpose(1, 2)
            a = torch.nn.functional.scaled_dot_product_attention(qq, kk, vv, scale=m.scale, enable_gqa=True)
            x = x + a.transpose(1, 2).reshape(B, S, -1) @ L["wo"].float().t()
            h = Fn.rms_norm(x, L["mlp_norm"], m.cfg.eps).float()
            gu = h @ L["wgu"].float().t()
            g, u = gu.chunk(2, -1)
            x = x + (torch.nn.functional.silu(g) * u) @ L["wd"].float().t()
        x = Fn.rms_norm(x, m.final_norm, m.cfg.eps).float()
        want.append((x[0].mean(0) @ eng.model.head_w.float().t() + eng.model.head_b).item())
    want = torch.tensor(want)
    assert torch.allclose(got, want, atol=0.05 * want.abs().max().item() + 1e-3), (got, want)
