"""FP8 (e4m3fn) KV cache on the CPU reference path: pages hold k / k_scale and v / v_scale,
the logits stay close to the bf16-cache model, copy-on-fork copies the raw bytes, and the
engine sizes twice the pages for the same bytes."""
import torch

from nv_genai_amd.models.config import llama_config
from nv_genai_amd.models.llama import AttnMeta, LlamaModel


def _logits(m, ids, kv_dtype, scales):
    T = ids.numel()
    m.allocate_kv_cache(8, 64, kv_dtype, scales)
    bt = torch.arange(8, dtype=torch.int32).unsqueeze(0)
    meta = AttnMeta(kind="prefill", slots=torch.arange(T - 1, dtype=torch.int32),
                    cu_q=torch.tensor([0, T - 1], dtype=torch.int32),
                    ctx_lens=torch.tensor([T - 1], dtype=torch.int32), block_tables=bt,
                    max_q_len=T - 1, max_ctx=T - 1)
    with torch.no_grad():
        m.forward(ids[:-1], torch.arange(T - 1, dtype=torch.int32), meta)
        meta = AttnMeta(kind="decode", slots=torch.tensor([T - 1], dtype=torch.int32),
                        cu_q=torch.tensor([0, 1], dtype=torch.int32),
                        ctx_lens=torch.tensor([T], dtype=torch.int32), block_tables=bt,
                        max_q_len=1, max_ctx=T)
        return m.logits(m.forward(ids[-1:], torch.tensor([T - 1], dtype=torch.int32), meta))[0].float()


def test_fp8_kv_logits_close_to_bf16():
    m = LlamaModel(llama_config("llama-tiny"), "cpu", seed=3)
    ids = torch.randint(3, m.cfg.vocab_size, (150,), generator=torch.Generator().manual_seed(1)).int()
    a = _logits(m, ids, "auto", (1.0, 1.0))
    for scales in ((1.0, 1.0), (0.25, 4.0)):
        b = _logits(m, ids, "fp8", scales)
        assert m.k_cache.dtype == torch.float8_e4m3fn
        assert torch.nn.functional.cosine_similarity(a, b, dim=0) > 0.999
        assert int(a.argmax()) == int(b.argmax())


def test_fp8_kv_scales_and_saturation():
    from nv_genai_amd.ops import reference as ref

    D, Hq, Hkv = 64, 2, 1
    qkv = torch.zeros(2, (Hq + 2 * Hkv) * D, dtype=torch.bfloat16)
    qkv[0, Hq * D] = 3.0            # k[0, 0]
    qkv[1, Hq * D] = 1000.0         # beyond e4m3's 448 after scaling: saturates
    qkv[0, (Hq + Hkv) * D] = -5.0   # v[0, 0]
    kc = torch.zeros(1, Hkv, 64, D, dtype=torch.uint8).view(torch.float8_e4m3fn)
    vc = torch.zeros(1, Hkv, D, 64, dtype=torch.uint8).view(torch.float8_e4m3fn)
    cs = ref.rope_cos_sin(16, D)
    ref.rope_cache_(qkv, torch.zeros(2, dtype=torch.int32), cs, torch.tensor([0, 1], dtype=torch.int32),
                    kc, vc, Hq, Hkv, D, kv_scales=(2.0, 0.5))
    assert float(kc[0, 0, 0, 0]) == 1.5 and float(kc[0, 0, 1, 0]) == 448.0
    assert float(vc[0, 0, 0, 0]) == -10.0


def test_engine_fp8_kv_pages_and_copy():
    from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine, SamplingParams

    e = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=4, max_batched_tokens=256, max_model_len=512,
                               kv_cache_blocks=16, kv_cache_dtype="fp8"), device="cpu")
    m = e.model
    assert m.kv_block_bytes(64, "fp8") * 2 == m.kv_block_bytes(64)
    out = e.generate([[5, 6, 7, 8] * 20], SamplingParams(temperature=0.0, max_tokens=5, ignore_eos=True))
    assert len(out[0].output_ids) == 5
    m.k_cache.view(torch.uint8)[:, 3] = 7
    m.copy_kv_blocks(torch.tensor([3]), torch.tensor([9]))
    assert torch.equal(m.k_cache.view(torch.uint8)[:, 9], m.k_cache.view(torch.uint8)[:, 3])
