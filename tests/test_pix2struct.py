"""DePlot / Pix2Struct engine (models/pix2struct.py) against transformers'
Pix2StructForConditionalGeneration and Pix2StructImageProcessorPil on CPU (fp32), plus the
hipGraph generation path and the model-server route on the GPU.

Parity: preprocessing (non-VQA mode; the VQA header is rendered with PIL's default font
instead of the checkpoint's Arial, so header pixels are parity unpinned), encoder states,
teacher-forced decoder logits and greedy generation, all on a random-init tiny config."""
import numpy as np
import pytest
import torch

from nv_genai_amd.models.pix2struct import (DePlot, Pix2StructModel, flatten_patches, pad_patches,
                                            pix2struct_config, relative_bucket, render_header)

transformers = pytest.importorskip("transformers")


def _hf_model(cfg, seed=0):
    from transformers import (Pix2StructConfig, Pix2StructForConditionalGeneration,
                              Pix2StructTextConfig, Pix2StructVisionConfig)

    vc = Pix2StructVisionConfig(hidden_size=cfg.v_hidden, patch_embed_hidden_size=cfg.patch_dim,
                                d_ff=cfg.v_ff, d_kv=cfg.v_dkv, num_attention_heads=cfg.v_heads,
                                num_hidden_layers=cfg.v_layers, seq_len=cfg.pos_table,
                                layer_norm_eps=cfg.eps)
    tc = Pix2StructTextConfig(hidden_size=cfg.t_hidden, d_ff=cfg.t_ff, d_kv=cfg.t_dkv, num_heads=cfg.t_heads,
                              num_layers=cfg.t_layers, vocab_size=cfg.vocab_size, dropout_rate=0.0,
                              relative_attention_num_buckets=cfg.rel_buckets,
                              relative_attention_max_distance=cfg.rel_max_distance)
    torch.manual_seed(seed)
    m = Pix2StructForConditionalGeneration(Pix2StructConfig(vision_config=vc.to_dict(), text_config=tc.to_dict(),
                                                            is_vqa=cfg.is_vqa))
    # HF's init leaves some weights tiny; widen everything so the comparison exercises them
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "layer_norm" in n or "layernorm" in n:
                p.copy_(1.0 + 0.1 * torch.randn_like(p))
            elif "relative_attention_bias" in n:
                p.normal_(0.0, 0.5)
            else:
                p.normal_(0.0, 0.08)
    return m.eval()


def _image(h, w, seed=0):
    rng = np.random.default_rng(seed)
    img = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
    img[h // 3: h // 2, :, 0] = 255                  # some structure beyond noise
    return img


def test_relative_bucket_matches_t5():
    from transformers.models.pix2struct.modeling_pix2struct import Pix2StructTextAttention

    rel = torch.arange(-300, 5)[None, :].repeat(2, 1)
    ref = Pix2StructTextAttention._relative_position_bucket(rel, bidirectional=False, num_buckets=32,
                                                            max_distance=128)
    assert torch.equal(relative_bucket(rel, 32, 128), ref)


@pytest.mark.parametrize("hw", [(37, 53), (120, 30), (16, 16)])
def test_flatten_patches_matches_hf_processor(hw):
    from transformers.models.pix2struct.image_processing_pil_pix2struct import Pix2StructImageProcessorPil

    cfg = pix2struct_config("pix2struct-tiny")
    img = _image(*hw)
    proc = Pix2StructImageProcessorPil(is_vqa=False, max_patches=cfg.max_patches,
                                       patch_size={"height": cfg.patch, "width": cfg.patch})
    ref = proc(images=img, return_tensors="pt")
    ours = flatten_patches(img, cfg.max_patches, cfg.patch)
    padded, mask = pad_patches(ours, cfg.max_patches)
    assert ours.shape[0] <= cfg.max_patches
    torch.testing.assert_close(padded, ref["flattened_patches"][0], atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(mask, ref["attention_mask"][0])


def test_encoder_decoder_and_generation_match_transformers():
    cfg = pix2struct_config("pix2struct-tiny")
    hf = _hf_model(cfg)
    ours = Pix2StructModel(cfg, device="cpu", dtype=torch.float32, weights=hf.state_dict())
    imgs = [_image(37, 53, 1), _image(60, 20, 2)]
    ps = [flatten_patches(im, cfg.max_patches, cfg.patch) for im in imgs]
    padded = torch.stack([pad_patches(p, cfg.max_patches)[0] for p in ps])
    mask = torch.stack([pad_patches(p, cfg.max_patches)[1] for p in ps])
    with torch.no_grad():
        enc_ref = hf.encoder(flattened_patches=padded, attention_mask=mask).last_hidden_state
    enc, cu = ours.encode(ps)
    for b, p in enumerate(ps):
        n = p.shape[0]
        torch.testing.assert_close(enc[int(cu[b]):int(cu[b]) + n], enc_ref[b, :n], atol=2e-4, rtol=2e-4)
    ids = torch.tensor([[0, 5, 17, 99, 3, 250], [0, 42, 42, 7, 1, 0]])
    with torch.no_grad():
        ref = hf(flattened_patches=padded, attention_mask=mask, decoder_input_ids=ids).logits
    got = ours.decode_logits(enc, cu, ids)
    torch.testing.assert_close(got, ref, atol=5e-4, rtol=5e-4)
    with torch.no_grad():
        gen = hf.generate(flattened_patches=padded, attention_mask=mask, max_new_tokens=12, do_sample=False)
    want = []
    for row in gen.tolist():
        row = row[1:]                                   # drop the decoder start token
        want.append(row[: row.index(cfg.eos_id)] if cfg.eos_id in row else row)
    assert ours.generate(ps, max_new_tokens=12, use_graph=False) == want


def test_state_dict_round_trip_and_deplot_describe():
    d = DePlot("pix2struct-tiny", device="cpu", seed=3)
    sd = d.model.state_dict()
    again = Pix2StructModel("pix2struct-tiny", device="cpu", dtype=torch.float32, weights=sd)
    for k, v in again.state_dict().items():
        assert torch.equal(v, sd[k]), k
    img = _image(40, 64, 5)
    hdr = render_header(img, DePlot.PROMPT)
    assert hdr.shape[1] >= img.shape[1] and hdr.shape[0] > img.shape[0]
    out = d.describe_batch([img, _image(20, 20, 6)], max_new_tokens=6)
    assert len(out) == 2 and all(isinstance(t, str) for t in out)


@pytest.mark.gpu
def test_deplot_gpu_matches_cpu_and_graph_replay():
    cfg = pix2struct_config("pix2struct-small")
    cpu = Pix2StructModel(cfg, device="cpu", dtype=torch.float32, seed=7)
    gpu = Pix2StructModel(cfg, device="cuda", dtype=torch.bfloat16, weights=cpu.state_dict())
    imgs = [_image(300, 400, 1), _image(128, 512, 2), _image(90, 90, 3)]
    ps = [flatten_patches(im, cfg.max_patches, cfg.patch) for im in imgs]
    enc_c, cu = cpu.encode(ps)
    enc_g, _ = gpu.encode(ps)
    row_cos = torch.nn.functional.cosine_similarity(enc_g.float().cpu(), enc_c, dim=1)
    assert float(row_cos.min()) > 0.99, row_cos.min()
    ids = torch.tensor([[0, 11, 12, 13], [0, 400, 2, 9], [0, 1, 0, 0]])
    lg = gpu.decode_logits(enc_g, cu.cuda(), ids.cuda()).cpu()
    lc = cpu.decode_logits(enc_c, cu, ids)
    cos = torch.nn.functional.cosine_similarity(lg.flatten(1), lc.flatten(1))
    assert bool((cos > 0.99).all()), cos
    # the hipGraph step and the eager step produce the same tokens on the same device
    a = gpu.generate(ps, max_new_tokens=24, use_graph=True)
    b = gpu.generate(ps, max_new_tokens=24, use_graph=False)
    assert a == b


def test_model_server_routes_deplot_requests():
    import base64
    import io

    from fastapi.testclient import TestClient
    from PIL import Image

    from nv_genai_amd.serving.model_server import create_app

    buf = io.BytesIO()
    Image.fromarray(_image(48, 64, 9)).save(buf, format="PNG")
    uri = "data:image/png;base64," + base64.b64encode(buf.getvalue()).decode()
    app = create_app(None, None, None, deplot=DePlot("pix2struct-tiny", device="cpu", seed=1))
    c = TestClient(app)
    assert "google/deplot" in [m["id"] for m in c.get("/v1/models").json()["data"]]
    msg = [{"role": "user", "content": [{"type": "text", "text": DePlot.PROMPT},
                                        {"type": "image_url", "image_url": {"url": uri}}]}]
    r = c.post("/v1/chat/completions", json={"model": "ai-google-deplot", "messages": msg, "max_tokens": 8})
    assert r.status_code == 200, r.text
    body = r.json()
    assert body["choices"][0]["message"]["role"] == "assistant"
    assert isinstance(body["choices"][0]["message"]["content"], str)
    s = c.post("/v1/chat/completions", json={"model": "google/deplot", "messages": msg, "max_tokens": 8,
                                             "stream": True})
    frames = [ln for ln in s.text.splitlines() if ln.startswith("data: ")]
    assert frames[-1] == "data: [DONE]" and len(frames) == 3
    bad = c.post("/v1/chat/completions", json={"model": "google/deplot",
                                               "messages": [{"role": "user", "content": "no image"}]})
    assert bad.status_code == 400


def test_generate_many_matches_per_batch_generation():
    d = DePlot("pix2struct-tiny", device="cpu", seed=4)
    imgs = [_image(30 + 7 * i, 50, i) for i in range(5)]
    many = d.generate_many(imgs, batch=2, max_new_tokens=5, threads=3)
    one = d.model.generate([d.patches(im) for im in imgs], max_new_tokens=5)
    assert many == one


def test_deplot_batcher_merges_concurrent_requests():
    from concurrent.futures import ThreadPoolExecutor

    from nv_genai_amd.models.pix2struct import DePlotBatcher

    d = DePlot("pix2struct-tiny", device="cpu", seed=2)
    imgs = [_image(30 + 5 * i, 40, 20 + i) for i in range(6)]
    want = [d.tok.decode(o[:3 + i]) for i, o in
            enumerate(d.model.generate([d.patches(im) for im in imgs], max_new_tokens=8))]
    b = DePlotBatcher(d, max_batch=8, max_delay_s=0.5)
    with ThreadPoolExecutor(6) as ex:
        got = list(ex.map(lambda i: b.describe(imgs[i], None, 3 + i), range(6)))
    assert got == want
    assert b.batches < 6


def test_local_vision_registry_serves_deplot_in_process(monkeypatch):
    import io

    from PIL import Image

    from nv_genai_amd.connectors import vision as vc

    monkeypatch.setattr(vc, "_LOCAL", {})
    monkeypatch.delenv("VLM_SERVER_URL", raising=False)
    monkeypatch.delenv("APP_VLM_SERVERURL", raising=False)
    monkeypatch.setenv("APP_VISION_LOCAL", "ai-google-deplot=pix2struct-tiny")
    buf = io.BytesIO()
    Image.fromarray(_image(40, 40, 3)).save(buf, format="PNG")
    c = vc.get_vision_client("ai-google-deplot")
    assert isinstance(c, vc.LocalDePlot)
    assert isinstance(c.describe(buf.getvalue(), DePlot.PROMPT, max_tokens=4), str)
    # names that are not registered keep the endpoint / heuristics path
    assert isinstance(vc.get_vision_client("ai-neva-22b"), vc.ImageHeuristics)
