"""Vision-language model (LLaVA / NeVA architecture) on the gfx950 kernel set.

The reference's multimodal pipeline sends every embedded image to hosted VLMs — NeVA-22B
("Describe this image in detail", then "is it a graph?") and DePlot (chart -> table) —
as an ``image_url`` data URI inside an OpenAI chat message
(RetrievalAugmentedGeneration/examples/multimodal_rag/llm/llm_client.py:37-42,
examples/multimodal_rag/vectorstore/custom_pdf_parser.py:29-71). This
module is the engine behind that contract: NeVA is a LLaVA-style model (a CLIP ViT image
encoder, an MLP projector into the LLM's embedding space, and a decoder LM that reads the
projected patch features in place of placeholder tokens).

* :class:`VisionTower` — CLIP ViT (pre-LN): patch embedding as one GEMM over unfolded
  patches, class token + learned positions, pre-LayerNorm, then encoder layers built from the
  same kernels as the BERT encoder: fused add+LayerNorm (``ops.add_layernorm``), biased
  hipBLASLt projections, bidirectional packed MFMA attention (``ops.varlen_attention``) and
  the quick-GELU MLP (``ops.bias_gelu_(..., "quick")``). Features come from layer
  ``feature_layer`` (LLaVA: the penultimate, CLS dropped); later layers are never run.
* projector — Linear -> GELU -> Linear (LLaVA-1.5 ``mlp2x_gelu``).
* :class:`VisionLanguageModel` — image preprocessing (PIL: shortest-side bicubic resize,
  centre crop, CLIP normalisation), prompt assembly with one placeholder token per patch,
  and generation through the continuous-batching :class:`LLMEngine`, which splices the
  image features into the prefill embeddings (``add_request(..., mm=...)``). Placeholder ids
  are derived from the image's content hash so the prefix cache can never reuse one image's
  KV for another.
"""
from __future__ import annotations

import hashlib
import io
import math
from dataclasses import dataclass, field, replace
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from .. import ops


@dataclass(frozen=True)
class VisionConfig:
    """CLIP ViT image encoder (defaults: ViT-L/14 at 336 px, LLaVA-1.5's tower)."""

    name: str = "clip-vit-l-14-336"
    image_size: int = 336
    patch: int = 14
    hidden: int = 1024
    layers: int = 24
    heads: int = 16
    ffn: int = 4096
    eps: float = 1e-5
    act: str = "quick"                 # CLIP quick_gelu
    feature_layer: int = -2            # hidden_states index LLaVA reads (penultimate layer)
    mean: tuple = (0.48145466, 0.4578275, 0.40821073)
    std: tuple = (0.26862954, 0.26130258, 0.27577711)

    @property
    def num_patches(self) -> int:
        return (self.image_size // self.patch) ** 2

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads


@dataclass(frozen=True)
class VLMConfig:
    name: str = "llava-1.5-7b"
    vision: VisionConfig = field(default_factory=VisionConfig)
    llm: str = "vicuna-7b"             # decoder preset (models/config.py)
    projector_act: str = "none"        # GELU form of the projector (LLaVA: exact erf GELU)


VLM_PRESETS: Dict[str, VLMConfig] = {
    # LLaVA-1.5-7B: CLIP ViT-L/14-336 + Vicuna-7B (Llama-2-7B dims)
    "llava-1.5-7b": VLMConfig(),
    # NeVA-22B stand-in (the reference's ``ai-neva-22b``): same architecture, CLIP ViT-L/14 at
    # 224 px and a 22B-class decoder of the Llama layout
    "neva-22b": VLMConfig(name="neva-22b", vision=VisionConfig(name="clip-vit-l-14-224", image_size=224),
                          llm="neva-22b-llm"),
    # small configs for tests
    "vlm-tiny": VLMConfig(name="vlm-tiny", vision=VisionConfig(name="vit-tiny", image_size=56, patch=14,
                                                               hidden=64, layers=3, heads=2, ffn=128),
                          llm="llama-tiny"),
    "vlm-small": VLMConfig(name="vlm-small", vision=VisionConfig(name="vit-small", image_size=224, patch=14,
                                                                 hidden=256, layers=4, heads=4, ffn=1024),
                           llm="llama-small"),
}


def vlm_config(name_or_cfg, **overrides) -> VLMConfig:
    cfg = VLM_PRESETS[name_or_cfg] if isinstance(name_or_cfg, str) else name_or_cfg
    return replace(cfg, **overrides) if overrides else cfg


class VisionTower:
    """CLIP ViT forward to the LLaVA feature layer (HF ``CLIPVisionModel`` weights)."""

    def __init__(self, cfg: VisionConfig, device="cuda", dtype=torch.bfloat16,
                 weights: Optional[Dict[str, torch.Tensor]] = None, seed: int = 0,
                 prefix: str = "model.vision_tower."):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        n_feat = cfg.layers + 1 + cfg.feature_layer if cfg.feature_layer < 0 else cfg.feature_layer
        if not 0 <= n_feat <= cfg.layers:
            raise ValueError(f"feature_layer {cfg.feature_layer} outside 0..{cfg.layers}")
        self.n_run = n_feat                   # hidden_states[k] = output of layer k - 1
        if weights is None:
            self._random_init(seed)
        else:
            self._load(weights, prefix)

    def _random_init(self, seed: int):
        c, dev, dt = self.cfg, self.device, self.dtype
        g = torch.Generator(device=dev).manual_seed(seed + 77)
        H = c.hidden

        def rnd(*shape, std=0.02):
            t = torch.empty(*shape, device=dev, dtype=dt)
            return t.normal_(0.0, std, generator=g)

        def ones(n):
            return torch.ones(n, device=dev, dtype=dt)

        def zeros(n):
            return torch.zeros(n, device=dev, dtype=dt)

        self.patch_w = rnd(H, 3 * c.patch * c.patch)
        self.cls = rnd(H)
        self.pos = rnd(c.num_patches + 1, H)
        self.pre_ln = (ones(H), zeros(H))
        self.layers = [{"ln1_g": ones(H), "ln1_b": zeros(H), "wqkv": rnd(3 * H, H), "bqkv": zeros(3 * H),
                        "wo": rnd(H, H), "bo": zeros(H), "ln2_g": ones(H), "ln2_b": zeros(H),
                        "w1": rnd(c.ffn, H), "b1": zeros(c.ffn), "w2": rnd(H, c.ffn), "b2": zeros(H)}
                       for _ in range(c.layers)]

    def _load(self, w: Dict[str, torch.Tensor], prefix: str):
        c, dev, dt = self.cfg, self.device, self.dtype

        def get(n):
            return w[prefix + n].to(dev, dt)

        self.patch_w = get("embeddings.patch_embedding.weight").reshape(c.hidden, -1).contiguous()
        self.cls = get("embeddings.class_embedding")
        self.pos = get("embeddings.position_embedding.weight")
        self.pre_ln = (get("pre_layrnorm.weight"), get("pre_layrnorm.bias"))
        self.layers = []
        for i in range(c.layers):
            p = f"encoder.layers.{i}."
            a = p + "self_attn."
            self.layers.append({
                "ln1_g": get(p + "layer_norm1.weight"), "ln1_b": get(p + "layer_norm1.bias"),
                "wqkv": torch.cat([get(a + "q_proj.weight"), get(a + "k_proj.weight"),
                                   get(a + "v_proj.weight")]).contiguous(),
                "bqkv": torch.cat([get(a + "q_proj.bias"), get(a + "k_proj.bias"), get(a + "v_proj.bias")]),
                "wo": get(a + "out_proj.weight"), "bo": get(a + "out_proj.bias"),
                "ln2_g": get(p + "layer_norm2.weight"), "ln2_b": get(p + "layer_norm2.bias"),
                "w1": get(p + "mlp.fc1.weight"), "b1": get(p + "mlp.fc1.bias"),
                "w2": get(p + "mlp.fc2.weight"), "b2": get(p + "mlp.fc2.bias"),
            })

    def state_dict(self, prefix: str = "model.vision_tower.") -> Dict[str, torch.Tensor]:
        """HF ``CLIPVisionModel`` names (inverse of ``_load``)."""
        c = self.cfg
        H = c.hidden
        out = {prefix + "embeddings.patch_embedding.weight": self.patch_w.reshape(H, 3, c.patch, c.patch),
               prefix + "embeddings.class_embedding": self.cls,
               prefix + "embeddings.position_embedding.weight": self.pos,
               prefix + "pre_layrnorm.weight": self.pre_ln[0], prefix + "pre_layrnorm.bias": self.pre_ln[1]}
        for i, L in enumerate(self.layers):
            p = prefix + f"encoder.layers.{i}."
            a = p + "self_attn."
            for j, n in enumerate(("q_proj", "k_proj", "v_proj")):
                out[a + n + ".weight"] = L["wqkv"][j * H:(j + 1) * H]
                out[a + n + ".bias"] = L["bqkv"][j * H:(j + 1) * H]
            out.update({a + "out_proj.weight": L["wo"], a + "out_proj.bias": L["bo"],
                        p + "layer_norm1.weight": L["ln1_g"], p + "layer_norm1.bias": L["ln1_b"],
                        p + "layer_norm2.weight": L["ln2_g"], p + "layer_norm2.bias": L["ln2_b"],
                        p + "mlp.fc1.weight": L["w1"], p + "mlp.fc1.bias": L["b1"],
                        p + "mlp.fc2.weight": L["w2"], p + "mlp.fc2.bias": L["b2"]})
        return out

    def patchify(self, pixels: torch.Tensor) -> torch.Tensor:
        """[B, 3, S, S] -> [B, P, 3 * p * p] (channel-major within a patch, like the conv weight)."""
        c = self.cfg
        B = pixels.shape[0]
        g = c.image_size // c.patch
        x = pixels.reshape(B, 3, g, c.patch, g, c.patch).permute(0, 2, 4, 1, 3, 5)
        return x.reshape(B, g * g, 3 * c.patch * c.patch)

    @torch.no_grad()
    def forward(self, pixels: torch.Tensor) -> torch.Tensor:
        """pixels [B, 3, S, S] (normalised) -> patch features [B, P, hidden] of the feature
        layer, CLS row dropped."""
        c = self.cfg
        B = pixels.shape[0]
        P, H = c.num_patches, c.hidden
        patches = self.patchify(pixels.to(self.device, self.dtype))
        emb = patches.reshape(B * P, -1) @ self.patch_w.t()                     # [B*P, H]
        x = torch.cat([self.cls.expand(B, 1, H), emb.view(B, P, H)], 1) + self.pos.unsqueeze(0)
        x = x.reshape(B * (P + 1), H).contiguous()
        x = ops.layernorm(x, self.pre_ln[0], self.pre_ln[1], c.eps)            # residual stream
        if self.n_run == 0:
            return x.view(B, P + 1, H)[:, 1:]
        cu = torch.arange(0, B + 1, device=self.device, dtype=torch.int32) * (P + 1)
        L0 = self.layers[0]
        h = ops.layernorm(x, L0["ln1_g"], L0["ln1_b"], c.eps)
        for li in range(self.n_run):
            L = self.layers[li]
            qkv = torch.addmm(L["bqkv"], h, L["wqkv"].t())
            a = ops.varlen_attention(qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:], cu, c.heads, c.heads,
                                     c.head_dim, P + 1, self.scale, causal=False)
            o = torch.addmm(L["bo"], a, L["wo"].t())
            h = ops.add_layernorm(x, o, L["ln2_g"], L["ln2_b"], c.eps)         # x += attention
            f = torch.addmm(L["b1"], h, L["w1"].t())
            ops.bias_gelu_(f, None, c.act)
            m = torch.addmm(L["b2"], f, L["w2"].t())
            if li + 1 < self.n_run:
                Ln = self.layers[li + 1]
                h = ops.add_layernorm(x, m, Ln["ln1_g"], Ln["ln1_b"], c.eps)   # x += MLP
            else:
                x = x + m
        return x.view(B, P + 1, H)[:, 1:]


class Projector:
    """LLaVA-1.5 ``mlp2x_gelu``: Linear -> GELU -> Linear into the LLM hidden size."""

    def __init__(self, d_in: int, d_out: int, device, dtype=torch.bfloat16, act: str = "none",
                 weights: Optional[Dict[str, torch.Tensor]] = None, seed: int = 0,
                 prefix: str = "model.multi_modal_projector."):
        self.act = act
        dev = torch.device(device)
        if weights is not None:
            get = lambda n: weights[prefix + n].to(dev, dtype)  # noqa: E731
            self.w1, self.b1 = get("linear_1.weight"), get("linear_1.bias")
            self.w2, self.b2 = get("linear_2.weight"), get("linear_2.bias")
        else:
            g = torch.Generator(device=dev).manual_seed(seed + 91)
            self.w1 = torch.empty(d_out, d_in, device=dev, dtype=dtype).normal_(0, 0.02, generator=g)
            self.w2 = torch.empty(d_out, d_out, device=dev, dtype=dtype).normal_(0, 0.02, generator=g)
            self.b1 = torch.zeros(d_out, device=dev, dtype=dtype)
            self.b2 = torch.zeros(d_out, device=dev, dtype=dtype)

    @torch.no_grad()
    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        y = torch.addmm(self.b1, x, self.w1.t())
        ops.bias_gelu_(y, None, self.act)
        return torch.addmm(self.b2, y, self.w2.t())


def preprocess_image(data: bytes, cfg: VisionConfig) -> torch.Tensor:
    """Image bytes (PNG / JPEG / GIF ...) -> normalised [3, S, S] float32: RGB, shortest side
    resized to S (bicubic), centre crop, CLIP mean / std (the CLIPImageProcessor recipe)."""
    from PIL import Image

    S = cfg.image_size
    im = Image.open(io.BytesIO(data)).convert("RGB")
    w, h = im.size
    s = S / min(w, h)
    im = im.resize((max(S, round(w * s)), max(S, round(h * s))), Image.BICUBIC)
    w, h = im.size
    left, top = (w - S) // 2, (h - S) // 2
    im = im.crop((left, top, left + S, top + S))
    x = torch.frombuffer(bytearray(im.tobytes()), dtype=torch.uint8).view(S, S, 3)
    x = x.permute(2, 0, 1).float() / 255.0
    mean = torch.tensor(cfg.mean).view(3, 1, 1)
    std = torch.tensor(cfg.std).view(3, 1, 1)
    return (x - mean) / std


def image_placeholder_ids(data: bytes, n: int, vocab: int) -> List[int]:
    """n placeholder ids derived from the image's content hash (prefix-cache safe)."""
    base = int.from_bytes(hashlib.sha1(data).digest()[:8], "little")
    return [(base + 7919 * i) % (vocab - 16) + 16 for i in range(n)]


def split_image_parts(content) -> Tuple[List[object], List[bytes]]:
    """Split an OpenAI chat message content into ordered parts — text strings, or the index of
    an image in the returned image list — and the image bytes (``image_url`` data URIs or raw
    ``{"type": "image", "image": bytes}`` parts)."""
    import base64

    if isinstance(content, str):
        return [content], []
    parts, images = [], []
    for p in content:
        if not isinstance(p, dict):
            continue
        t = p.get("type", "text")
        if t == "text":
            parts.append(p.get("text", ""))
        elif t in ("image_url", "image"):
            if t == "image":
                data = p["image"]
            else:
                url = p["image_url"]["url"] if isinstance(p["image_url"], dict) else p["image_url"]
                if not url.startswith("data:"):
                    raise ValueError("only data: URIs are accepted for images (no network access)")
                data = base64.b64decode(url.split(",", 1)[1])
            parts.append(len(images))
            images.append(data)
    return parts, images


class VisionLanguageModel:
    """Tower + projector + a continuous-batching decoder engine.

    ``submit(messages)`` takes OpenAI chat messages whose content may hold ``image_url`` parts
    (data URIs) or raw ``{"type": "image", "image": bytes}`` parts; the prompt follows the
    LLaVA-1.5 conversation format ("USER: <image>\\n... ASSISTANT:"), every image expanding to
    one placeholder per patch whose embeddings the engine replaces with the projected
    features."""

    def __init__(self, cfg, device=None, engine=None, engine_cfg=None, weights=None, seed: int = 0,
                 pctx=None):
        from ..engine.llm_engine import EngineConfig, LLMEngine

        self.cfg = vlm_config(cfg)
        if engine is None:
            ecfg = engine_cfg or EngineConfig(model=self.cfg.llm)
            llm_w = None
            if weights is not None:
                llm_w = {k.replace("model.language_model.", "model."): v for k, v in weights.items()
                         if k.startswith("model.language_model.")}
                if "lm_head.weight" in weights:
                    llm_w["lm_head.weight"] = weights["lm_head.weight"]
            engine = LLMEngine(ecfg, device=device, weights=llm_w, pctx=pctx)
        self.engine = engine
        self.device = engine.device
        H_llm = engine.mcfg.hidden
        v = self.cfg.vision
        self.tower = VisionTower(v, self.device, weights=weights, seed=seed)
        self.projector = Projector(v.hidden, H_llm, self.device, act=self.cfg.projector_act,
                                   weights=weights, seed=seed)

    # ---------------------------------------------------------------- images
    @torch.no_grad()
    def encode_images(self, pixels: torch.Tensor) -> torch.Tensor:
        """[B, 3, S, S] -> projected features [B, P, H_llm] (bf16, on the engine device).
        Runs on request threads: its library GEMMs hold ``capture_guard`` (no graph capture of
        another thread is in progress while they launch)."""
        from ..utils.runtime import capture_guard

        with capture_guard():
            f = self.tower.forward(pixels)
            B, P, Hv = f.shape
            return self.projector(f.reshape(B * P, Hv).contiguous()).view(B, P, -1)

    def _images_of(self, content) -> Tuple[List[object], List[bytes]]:
        return split_image_parts(content)

    def image_features(self, datas: Sequence[bytes], batch: int = 32, threads: int = 8) -> Dict[bytes, torch.Tensor]:
        """Projected features of many images at once: decode / resize / normalise on host
        threads (PIL drops the GIL), then the CLIP tower and projector in batches of ``batch``
        images (one packed forward instead of one per request). Keyed by the image bytes."""
        from concurrent.futures import ThreadPoolExecutor

        uniq = list(dict.fromkeys(datas))
        if not uniq:
            return {}
        with ThreadPoolExecutor(max(1, min(threads, len(uniq)))) as ex:
            pix = list(ex.map(lambda d: preprocess_image(d, self.cfg.vision), uniq))
        out: Dict[bytes, torch.Tensor] = {}
        for i in range(0, len(uniq), batch):
            f = self.encode_images(torch.stack(pix[i:i + batch]))
            for j, d in enumerate(uniq[i:i + batch]):
                out[d] = f[j]
        return out

    def build_request(self, messages: Sequence[dict], features: Optional[Dict[bytes, torch.Tensor]] = None):
        """-> (prompt ids, [(offset, features)]) in the LLaVA-1.5 conversation format.
        ``features``: precomputed image features (:meth:`image_features`) to use instead of
        running the tower for this request."""
        tok = self.engine.tok
        vocab = self.engine.mcfg.vocab_size
        P = self.cfg.vision.num_patches
        ids = [tok.bos_id]
        imgs: List[Tuple[int, bytes]] = []
        system = ""
        for m in messages:
            role = m.get("role", "user")
            parts, images = self._images_of(m.get("content", ""))
            if role == "system":
                system = "".join(x for x in parts if isinstance(x, str)).strip() + " "
                continue
            ids += tok.encode((system if system else "") + ("USER: " if role == "user" else "ASSISTANT: "))
            system = ""
            for x in parts:
                if isinstance(x, str):
                    ids += tok.encode(x)
                else:
                    data = images[x]
                    imgs.append((len(ids), data))
                    ids += image_placeholder_ids(data, P, vocab)
                    ids += tok.encode("\n")
            ids += tok.encode(" ") if role == "user" else [tok.eot_id]
        ids += tok.encode("ASSISTANT:")
        mm = []
        if imgs:
            if features is not None and all(d in features for _, d in imgs):
                mm = [(off, features[d]) for off, d in imgs]
            else:
                pix = torch.stack([preprocess_image(d, self.cfg.vision) for _, d in imgs])
                feats = self.encode_images(pix)
                mm = [(off, feats[i]) for i, (off, _) in enumerate(imgs)]
        return ids, mm

    def submit(self, messages: Sequence[dict], params=None, on_token=None, features=None):
        ids, mm = self.build_request(messages, features)
        return self.engine.add_request(ids, params, on_token=on_token, mm=mm)

    def generate(self, messages_list: Sequence[Sequence[dict]], params=None):
        """Many chats at once: every image's features come from one batched tower pass."""
        datas = [d for msgs in messages_list for m in msgs
                 for d in split_image_parts(m.get("content", ""))[1]]
        feats = self.image_features(datas) if len(datas) > 1 else None
        reqs = [self.submit(m, params, features=feats) for m in messages_list]
        self.engine.run_until_done(reqs)
        return reqs

    def describe(self, image: bytes, prompt: str = "Describe this image in detail", max_tokens: int = 256,
                 **steer) -> str:
        """The ``VisionClient.describe`` contract of connectors/vision.py, served locally."""
        from ..engine.llm_engine import SamplingParams

        labels = ",".join(f"{k}:{v}" for k, v in steer.items())
        text = prompt + (f" [labels: {labels}]" if labels else "")
        r = self.generate([[{"role": "user", "content": [{"type": "text", "text": text},
                                                         {"type": "image", "image": image}]}]],
                          SamplingParams(temperature=0.2, top_p=0.7, max_tokens=max_tokens))[0]
        return r.text
