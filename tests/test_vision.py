"""Vision-language model (LLaVA / NeVA architecture): CLIP ViT tower +
projector + decoder with image features spliced into the prefill embeddings.

Parity is pinned against transformers' ``LlavaForConditionalGeneration`` (random weights of a
tiny config, CPU): our tower, projector and decoder load the HF state dict and must reproduce
HF's logits. The end-to-end tests run ``VisionLanguageModel`` through the continuous-batching
engine with real PNG bytes (PIL)."""
import base64
import io

import pytest
import torch

from nv_genai_amd.models.vision import (Projector, VisionConfig, VisionLanguageModel, VisionTower,
                                        image_placeholder_ids, preprocess_image, vlm_config)

transformers = pytest.importorskip("transformers")


def _png(seed=0, size=(40, 30)):
    from PIL import Image

    g = torch.Generator().manual_seed(seed)
    arr = (torch.rand(size[1], size[0], 3, generator=g) * 255).to(torch.uint8).numpy()
    buf = io.BytesIO()
    Image.fromarray(arr).save(buf, format="PNG")
    return buf.getvalue()


def test_llava_matches_transformers():
    from nv_genai_amd.models.config import llama_config
    from nv_genai_amd.models.llama import AttnMeta, LlamaModel

    lc = llama_config("llama-tiny")
    vc = transformers.CLIPVisionConfig(hidden_size=64, intermediate_size=128, num_hidden_layers=3,
                                       num_attention_heads=2, image_size=56, patch_size=14,
                                       hidden_act="quick_gelu", layer_norm_eps=1e-5)
    tc = transformers.LlamaConfig(vocab_size=lc.vocab_size, hidden_size=lc.hidden, intermediate_size=lc.ffn,
                                  num_hidden_layers=lc.layers, num_attention_heads=lc.heads,
                                  num_key_value_heads=lc.kv_heads, head_dim=lc.head_dim,
                                  rope_parameters={"rope_theta": lc.rope_theta, "rope_type": "default"},
                                  rms_norm_eps=lc.eps, max_position_embeddings=lc.max_position,
                                  bos_token_id=1, eos_token_id=2, pad_token_id=0)
    img_tok = 32000
    cfg = transformers.LlavaConfig(vision_config=vc, text_config=tc, image_token_id=img_tok,
                                   projector_hidden_act="gelu", vision_feature_layer=-2,
                                   vision_feature_select_strategy="default")
    torch.manual_seed(0)
    hf = transformers.LlavaForConditionalGeneration(cfg).eval()
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for n, p in hf.named_parameters():
            if "norm" in n and n.endswith("weight"):
                p.copy_(1.0 + 0.1 * torch.randn(p.shape, generator=g))
            elif n.endswith("bias"):
                p.copy_(0.02 * torch.randn(p.shape, generator=g))
            else:
                p.copy_(0.05 * torch.randn(p.shape, generator=g))
    sd = {k: v.detach().clone() for k, v in hf.state_dict().items()}
    hf = hf.to(torch.bfloat16)

    vcfg = VisionConfig(name="t", image_size=56, patch=14, hidden=64, layers=3, heads=2, ffn=128)
    tower = VisionTower(vcfg, "cpu", weights=sd)
    proj = Projector(64, lc.hidden, "cpu", weights=sd)
    llm_w = {k.replace("model.language_model.", "model."): v for k, v in sd.items() if "language_model" in k}
    llm_w["lm_head.weight"] = sd["lm_head.weight"]
    dec = LlamaModel(lc, "cpu", weights=llm_w)
    dec.allocate_kv_cache(2, 64)

    pix = preprocess_image(_png(3), vcfg).unsqueeze(0)
    P = vcfg.num_patches
    ids = torch.tensor([1, 57, 99] + [img_tok] * P + [400, 401, 402])
    with torch.no_grad():
        want = hf(input_ids=ids.unsqueeze(0), pixel_values=pix.to(torch.bfloat16)).logits[0].float()
        feats = proj(tower.forward(pix).reshape(P, -1))
        T = ids.numel()
        meta = AttnMeta(kind="prefill", slots=torch.arange(T, dtype=torch.int32),
                        cu_q=torch.tensor([0, T], dtype=torch.int32), ctx_lens=torch.tensor([T], dtype=torch.int32),
                        block_tables=torch.arange(2, dtype=torch.int32).unsqueeze(0), max_q_len=T, max_ctx=T)
        h = dec.forward(ids.int(), torch.arange(T, dtype=torch.int32), meta,
                        embed_override=(torch.arange(3, 3 + P), feats))
        got = dec.logits(h).float()
    cos = torch.nn.functional.cosine_similarity(got[-1], want[-1], dim=0).item()
    err = ((got - want).norm() / want.norm()).item()
    assert cos > 0.999 and err < 0.05, (cos, err)
    # bf16 near-ties of the random tiny model may flip an argmax or two between the op sets
    agree = (got.argmax(-1) == want.argmax(-1)).float().mean().item()
    assert agree >= 0.9 and got[-1].argmax() == want[-1].argmax(), agree


def test_vlm_engine_describes_images_and_prefix_cache_is_image_safe():
    from nv_genai_amd.engine.llm_engine import EngineConfig, SamplingParams

    vlm = VisionLanguageModel("vlm-tiny", device="cpu",
                              engine_cfg=EngineConfig(model="llama-tiny", max_num_seqs=4, max_batched_tokens=512,
                                                      max_model_len=1024, kv_cache_blocks=64, use_graphs=False))
    a, b = _png(1, (200, 120)), _png(2, (64, 64))
    P = vlm.cfg.vision.num_patches
    ids_a, mm_a = vlm.build_request([{"role": "user", "content": [
        {"type": "text", "text": "Describe this image in detail"},
        {"type": "image_url", "image_url": {"url": "data:image/png;base64," + base64.b64encode(a).decode()}}]}])
    assert len(mm_a) == 1 and mm_a[0][1].shape == (P, vlm.engine.mcfg.hidden)
    off = mm_a[0][0]
    assert ids_a[off:off + P] == image_placeholder_ids(a, P, vlm.engine.mcfg.vocab_size)
    assert image_placeholder_ids(a, P, 32768) != image_placeholder_ids(b, P, 32768)
    p = SamplingParams(temperature=0.0, max_tokens=5, ignore_eos=True)
    msgs = lambda img: [{"role": "user", "content": [{"type": "text", "text": "what is shown?"},  # noqa: E731
                                                      {"type": "image", "image": img}]}]
    r1, r2 = vlm.generate([msgs(a), msgs(b)], p)
    assert len(r1.output_ids) == 5 and len(r2.output_ids) == 5
    # the same image again: identical greedy output (its KV may come from the prefix cache)
    r3 = vlm.generate([msgs(a)], p)[0]
    assert r3.output_ids == r1.output_ids
    # features matter: the same prompt ids with another image's features decode differently
    ids_b, mm_b = vlm.build_request(msgs(b))
    ids_a2, mm_a2 = vlm.build_request(msgs(a))
    fa = vlm.engine.add_request(ids_a2, p, mm=mm_a2)
    fx = vlm.engine.add_request(ids_a2, p, mm=[(mm_a2[0][0], mm_b[0][1] * 3.0)])
    vlm.engine.run_until_done([fa, fx])
    assert fa.output_ids == r1.output_ids
    assert isinstance(vlm.describe(a, max_tokens=4), str)


def test_model_server_serves_vision_chat_and_vision_client(monkeypatch):
    """``/v1/chat/completions`` with an ``image_url`` data URI is served by the hosted VLM;
    the reference-style ``VisionClient`` (connectors/vision.py, the NeVA client of the
    multimodal example) talks to it over real HTTP."""
    import socket
    import threading
    import time

    import uvicorn
    from fastapi.testclient import TestClient

    from nv_genai_amd.connectors.vision import VisionClient, get_vision_client
    from nv_genai_amd.engine.llm_engine import EngineConfig
    from nv_genai_amd.serving.engine_service import EngineService
    from nv_genai_amd.serving.model_server import create_app

    vlm = VisionLanguageModel("vlm-tiny", device="cpu",
                              engine_cfg=EngineConfig(model="llama-tiny", max_num_seqs=4, max_batched_tokens=512,
                                                      max_model_len=1024, kv_cache_blocks=64, use_graphs=False))
    vsvc = EngineService(vlm.engine, name="vlm")
    app = create_app(None, None, None, vlm=vlm, vlm_service=vsvc, vlm_name="ai-neva-22b")
    img = _png(5, (90, 70))
    body = {"model": "ai-neva-22b", "max_tokens": 6, "temperature": 0.1, "messages": [{"role": "user", "content": [
        {"type": "text", "text": "Describe this image in detail"},
        {"type": "image_url", "image_url": {"url": "data:image/png;base64," + base64.b64encode(img).decode()}}]}]}
    with TestClient(app) as c:
        assert "ai-neva-22b" in [m["id"] for m in c.get("/v1/models").json()["data"]]
        r = c.post("/v1/chat/completions", json=body)
        assert r.status_code == 200, r.text
        assert r.json()["usage"]["prompt_tokens"] > vlm.cfg.vision.num_patches
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    srv = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="error"))
    t = threading.Thread(target=srv.run, daemon=True)
    t.start()
    try:
        for _ in range(200):
            if srv.started:
                break
            time.sleep(0.05)
        monkeypatch.setenv("VLM_SERVER_URL", f"http://127.0.0.1:{port}")
        client = get_vision_client("ai-neva-22b")
        assert isinstance(client, VisionClient)
        out = client.describe(img, "Describe this image in detail", creativity=0, quality=9)
        assert isinstance(out, str)
    finally:
        srv.should_exit = True
        t.join(timeout=5)
        vsvc.shutdown()
