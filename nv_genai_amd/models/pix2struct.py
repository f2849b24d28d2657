"""DePlot / Pix2Struct chart-to-table model on the gfx950 kernel set.

The reference's multimodal ingestion sends every chart it finds to DePlot with the prompt
"Generate underlying data table of the figure below:" and feeds the linearised table to the
LLM (RetrievalAugmentedGeneration/examples/multimodal_rag/vectorstore/custom_pdf_parser.py:55-71,
``process_graph``; notebooks/04 uses the same call; BASELINE.json configs[4]). DePlot is a
Pix2Struct model — an image-to-text encoder-decoder — so it gets its own engine here instead of
riding on the LLaVA-style VLM (models/vision.py):

* **Preprocessing** (:func:`flatten_patches`): the aspect-ratio-preserving Pix2Struct recipe —
  per-image standardisation, bilinear (antialiased) resize to the largest grid of 16x16 patches
  that fits ``max_patches``, patches flattened channel-last with 1-based (row, column) ids in
  front. In VQA mode (DePlot) the question is rendered as a header above the image
  (:func:`render_header`).
* **Encoder** (:meth:`Pix2StructModel.encode`): patch projection + learned row / column
  embeddings, then T5-style pre-norm layers — RMSNorm (``ops.rmsnorm`` / fused
  ``ops.add_rmsnorm``), one fused QKV GEMM, packed variable-length bidirectional MFMA
  attention (``ops.varlen_attention``: only real patches are packed, so padding costs nothing)
  with the unscaled T5 dot product, and the gated-GELU MLP (one fused wi_0|wi_1 GEMM +
  ``ops.gelu_tanh_mul``).
* **Decoder** (:meth:`Pix2StructModel.decode_logits` / :meth:`Pix2StructModel.generate`): T5 decoder layers (causal self-attention with the
  bucketed relative position bias of layer 0 shared by every layer, cross-attention to the
  encoder rows, gated-GELU MLP). Generation is batched over images: every layer's cross K/V
  are computed once in a single GEMM into 64-token KV pages, so cross-attention runs on the
  paged non-causal MFMA attention kernel (``ops.prefill_attention_paged``, each image's patch
  count as its context length); the self-attention KV cache is a static buffer, and on a
  GPU the whole decode step — embedding, 12 layers, LM head, greedy pick, cache write — is
  captured once into a hipGraph and replayed per token (the step index lives on the device, so
  the relative-bias row and the cache slot are gathered by the kernels, not by the host).

Weights use the HF ``Pix2StructForConditionalGeneration`` names (``load_state_dict`` /
``state_dict``); ``tests/test_pix2struct.py`` checks preprocessing, encoder states, teacher-
forced logits and greedy generation against transformers on CPU.
"""
from __future__ import annotations

import io
import math
import textwrap
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..utils.runtime import capture_guard
from .. import ops


@dataclass(frozen=True)
class Pix2StructConfig:
    name: str = "deplot"
    # vision encoder (pix2struct-base, DePlot's backbone)
    patch: int = 16
    max_patches: int = 2048
    v_hidden: int = 768
    v_layers: int = 12
    v_heads: int = 12
    v_dkv: int = 64
    v_ff: int = 2048
    pos_table: int = 4096              # rows of the row / column embedding tables
    # text decoder
    t_hidden: int = 768
    t_layers: int = 12
    t_heads: int = 12
    t_ff: int = 2048
    vocab_size: int = 50244
    rel_buckets: int = 32
    rel_max_distance: int = 128
    eps: float = 1e-6
    decoder_start_id: int = 0
    eos_id: int = 1
    pad_id: int = 0
    is_vqa: bool = True                # DePlot renders its prompt as an image header

    @property
    def patch_dim(self) -> int:
        return 3 * self.patch * self.patch

    @property
    def t_dkv(self) -> int:
        return self.t_hidden // self.t_heads


PIX2STRUCT_PRESETS: Dict[str, Pix2StructConfig] = {
    "deplot": Pix2StructConfig(),
    "pix2struct-tiny": Pix2StructConfig(name="pix2struct-tiny", patch=4, max_patches=64, v_hidden=64,
                                        v_layers=2, v_heads=4, v_dkv=16, v_ff=96, pos_table=64,
                                        t_hidden=64, t_layers=2, t_heads=4, t_ff=96, vocab_size=300),
    "pix2struct-small": Pix2StructConfig(name="pix2struct-small", patch=16, max_patches=512, v_hidden=256,
                                         v_layers=4, v_heads=4, v_dkv=64, v_ff=512, pos_table=512,
                                         t_hidden=256, t_layers=4, t_heads=4, t_ff=512, vocab_size=4096),
}


def pix2struct_config(name_or_cfg) -> Pix2StructConfig:
    return PIX2STRUCT_PRESETS[name_or_cfg] if isinstance(name_or_cfg, str) else name_or_cfg


# ----------------------------------------------------------------------------- preprocessing
def _to_rgb_array(image) -> np.ndarray:
    """bytes / PIL image / HWC uint8 array -> HWC uint8 RGB array."""
    if isinstance(image, np.ndarray):
        return image
    from PIL import Image

    if isinstance(image, (bytes, bytearray)):
        image = Image.open(io.BytesIO(image))
    return np.asarray(image.convert("RGB"))


def render_header(image, header: str, font_size: int = 36) -> np.ndarray:
    """Pix2Struct VQA input: ``header`` rendered (80-column wrap, 5 px padding, black on white)
    above the image, both scaled to the wider of the two. The reference model was trained with
    Arial; this renders with PIL's default font (no font files are downloaded here), so the
    header pixels — not the layout — differ from the HF processor."""
    from PIL import Image, ImageDraw, ImageFont

    img = Image.fromarray(_to_rgb_array(image))
    try:
        font = ImageFont.load_default(size=font_size)
    except TypeError:                     # PIL without scalable default fonts
        font = ImageFont.load_default()
    text = "\n".join(textwrap.TextWrapper(width=80).wrap(text=header))
    probe = ImageDraw.Draw(Image.new("RGB", (1, 1), "white"))
    _, _, tw, th = probe.textbbox((0, 0), text, font=font)
    pad = 5
    head = Image.new("RGB", (tw + 2 * pad, th + 2 * pad), "white")
    ImageDraw.Draw(head).text((pad, pad), text, fill="black", font=font)
    W = max(head.width, img.width)
    H_img = int(img.height * (W / img.width))
    H_head = int(head.height * (W / head.width))
    out = Image.new("RGB", (W, H_img + H_head), "white")
    out.paste(head.resize((W, H_head)), (0, 0))
    out.paste(img.resize((W, H_img)), (0, H_head))
    return np.asarray(out)


def flatten_patches(image, max_patches: int, patch: int = 16, normalize: bool = True,
                    device=None) -> torch.Tensor:
    """One image -> its real patches [rows * cols, 2 + 3 * patch^2] float32 (row id, column id,
    then the channel-last patch pixels); ``pad_patches`` pads to ``max_patches`` rows as the HF
    processor does. Same arithmetic as transformers' ``Pix2StructImageProcessorPil``:
    standardise with the image's mean / population std (std floored at 1 / sqrt(numel)), then
    resize (bilinear, antialiased) to the largest patch grid with rows * cols <= max_patches.
    ``device``: run the standardise / resize / patchify on that device (the uint8 pixels are
    uploaded once; on a GPU this takes the per-pixel work off the host)."""
    x = torch.from_numpy(np.ascontiguousarray(_to_rgb_array(image).transpose(2, 0, 1)))   # [3, h, w] u8
    if device is not None:
        x = x.to(device, non_blocking=True)
    x = x.float()
    if normalize:
        std = x.std(correction=0)
        x = (x - x.mean()) / torch.clamp(std, min=1.0 / math.sqrt(x.numel()))
    _, h, w = x.shape
    scale = math.sqrt(max_patches * (patch / h) * (patch / w))
    rows = max(min(int(scale * h / patch), max_patches), 1)
    cols = max(min(int(scale * w / patch), max_patches), 1)
    x = torch.nn.functional.interpolate(x[None], size=(rows * patch, cols * patch), mode="bilinear",
                                        align_corners=False, antialias=True)[0]
    p = x.reshape(3, rows, patch, cols, patch).permute(1, 3, 2, 4, 0).reshape(rows * cols, -1)
    r = torch.arange(rows, dtype=torch.float32, device=x.device).repeat_interleave(cols) + 1
    c = torch.arange(cols, dtype=torch.float32, device=x.device).repeat(rows) + 1
    return torch.cat([r[:, None], c[:, None], p], 1)


def pad_patches(p: torch.Tensor, max_patches: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """[n, D] -> ([max_patches, D] zero-padded, attention mask [max_patches])."""
    out = torch.zeros(max_patches, p.shape[1], dtype=p.dtype)
    out[: p.shape[0]] = p
    mask = torch.zeros(max_patches)
    mask[: p.shape[0]] = 1.0
    return out, mask


# ----------------------------------------------------------------------------- model
def relative_bucket(rel: torch.Tensor, num_buckets: int, max_distance: int) -> torch.Tensor:
    """T5 causal relative-position bucket of ``rel = key - query`` (bidirectional=False):
    exact buckets for the nearest num_buckets / 2 distances, log-spaced up to max_distance."""
    n = torch.clamp(-rel, min=0)
    max_exact = num_buckets // 2
    large = max_exact + (torch.log(n.float().clamp(min=1) / max_exact) / math.log(max_distance / max_exact)
                         * (num_buckets - max_exact)).long()
    large = torch.clamp(large, max=num_buckets - 1)
    return torch.where(n < max_exact, n, large)


class Pix2StructModel:
    """Encoder + decoder weights and the forward passes. ``weights``: HF state dict."""

    def __init__(self, cfg="deplot", device="cuda", dtype=torch.bfloat16,
                 weights: Optional[Dict[str, torch.Tensor]] = None, seed: int = 0):
        self.cfg = c = pix2struct_config(cfg)
        self.device = torch.device(device)
        self.dtype = dtype
        if c.t_heads * c.t_dkv != c.t_hidden:
            raise ValueError("text heads x head dim must equal the text hidden size")
        if weights is None:
            weights = self._random_state(seed)
        self.load_state_dict(weights)
        self._graphs: Dict[tuple, tuple] = {}

    # -- weights
    def _random_state(self, seed: int) -> Dict[str, torch.Tensor]:
        c = self.cfg
        g = torch.Generator().manual_seed(seed + 4242)

        def rnd(*shape, std=0.02):
            return torch.empty(*shape).normal_(0.0, std, generator=g)

        w = {"encoder.embeddings.patch_projection.weight": rnd(c.v_hidden, c.patch_dim),
             "encoder.embeddings.patch_projection.bias": torch.zeros(c.v_hidden),
             "encoder.embeddings.row_embedder.weight": rnd(c.pos_table, c.v_hidden),
             "encoder.embeddings.column_embedder.weight": rnd(c.pos_table, c.v_hidden),
             "encoder.layernorm.weight": torch.ones(c.v_hidden),
             "decoder.embed_tokens.weight": rnd(c.vocab_size, c.t_hidden, std=1.0),
             "decoder.final_layer_norm.weight": torch.ones(c.t_hidden),
             "decoder.lm_head.weight": rnd(c.vocab_size, c.t_hidden),
             "decoder.layer.0.self_attention.attention.relative_attention_bias.weight":
                 rnd(c.rel_buckets, c.t_heads, std=0.5)}
        inner = c.v_heads * c.v_dkv
        for i in range(c.v_layers):
            p = f"encoder.encoder.layer.{i}."
            for n in ("query", "key", "value"):
                w[p + f"attention.{n}.weight"] = rnd(inner, c.v_hidden)
            w[p + "attention.output.weight"] = rnd(c.v_hidden, inner)
            w[p + "mlp.wi_0.weight"] = rnd(c.v_ff, c.v_hidden)
            w[p + "mlp.wi_1.weight"] = rnd(c.v_ff, c.v_hidden)
            w[p + "mlp.wo.weight"] = rnd(c.v_hidden, c.v_ff)
            w[p + "pre_attention_layer_norm.weight"] = torch.ones(c.v_hidden)
            w[p + "pre_mlp_layer_norm.weight"] = torch.ones(c.v_hidden)
        H = c.t_hidden
        for i in range(c.t_layers):
            p = f"decoder.layer.{i}."
            for blk in ("self_attention", "encoder_decoder_attention"):
                for n in ("query", "key", "value", "output"):
                    w[p + f"{blk}.attention.{n}.weight"] = rnd(H, H)
                w[p + f"{blk}.layer_norm.weight"] = torch.ones(H)
            w[p + "mlp.DenseReluDense.wi_0.weight"] = rnd(c.t_ff, H)
            w[p + "mlp.DenseReluDense.wi_1.weight"] = rnd(c.t_ff, H)
            w[p + "mlp.DenseReluDense.wo.weight"] = rnd(H, c.t_ff)
            w[p + "mlp.layer_norm.weight"] = torch.ones(H)
        return w

    def load_state_dict(self, w: Dict[str, torch.Tensor]) -> None:
        c, dev, dt = self.cfg, self.device, self.dtype

        def get(n):
            return w[n].to(dev, dt).contiguous()

        e = "encoder."
        self.patch_w = get(e + "embeddings.patch_projection.weight")
        self.patch_b = get(e + "embeddings.patch_projection.bias")
        self.row_emb = get(e + "embeddings.row_embedder.weight")
        self.col_emb = get(e + "embeddings.column_embedder.weight")
        self.enc_norm = get(e + "layernorm.weight")
        self.enc_layers = []
        for i in range(c.v_layers):
            p = e + f"encoder.layer.{i}."
            a = p + "attention."
            self.enc_layers.append({
                "ln1": get(p + "pre_attention_layer_norm.weight"), "ln2": get(p + "pre_mlp_layer_norm.weight"),
                "wqkv": torch.cat([get(a + "query.weight"), get(a + "key.weight"), get(a + "value.weight")]),
                "wo": get(a + "output.weight"),
                "wi": torch.cat([get(p + "mlp.wi_0.weight"), get(p + "mlp.wi_1.weight")]),
                "wout": get(p + "mlp.wo.weight")})
        d = "decoder."
        self.embed = get(d + "embed_tokens.weight")
        self.dec_norm = get(d + "final_layer_norm.weight")
        self.lm_head = get(d + "lm_head.weight")
        self.rel_bias = w[d + "layer.0.self_attention.attention.relative_attention_bias.weight"].to(dev, torch.float32)
        self.dec_layers = []
        for i in range(c.t_layers):
            p = d + f"layer.{i}."
            s, x = p + "self_attention.", p + "encoder_decoder_attention."
            self.dec_layers.append({
                "ln_s": get(s + "layer_norm.weight"), "ln_x": get(x + "layer_norm.weight"),
                "ln_f": get(p + "mlp.layer_norm.weight"),
                "wqkv": torch.cat([get(s + "attention.query.weight"), get(s + "attention.key.weight"),
                                   get(s + "attention.value.weight")]),
                "wo": get(s + "attention.output.weight"),
                "wq_x": get(x + "attention.query.weight"), "wo_x": get(x + "attention.output.weight"),
                "wi": torch.cat([get(p + "mlp.DenseReluDense.wi_0.weight"), get(p + "mlp.DenseReluDense.wi_1.weight")]),
                "wout": get(p + "mlp.DenseReluDense.wo.weight")})
        # every layer's cross-attention K and V projections, one GEMM over the encoder rows
        self.w_xkv = torch.cat([torch.cat([get(d + f"layer.{i}.encoder_decoder_attention.attention.key.weight"),
                                           get(d + f"layer.{i}.encoder_decoder_attention.attention.value.weight")])
                                for i in range(c.t_layers)])
        self._graphs = {}

    def state_dict(self) -> Dict[str, torch.Tensor]:
        """HF ``Pix2StructForConditionalGeneration`` names (inverse of ``load_state_dict``)."""
        c = self.cfg
        w = {"encoder.embeddings.patch_projection.weight": self.patch_w,
             "encoder.embeddings.patch_projection.bias": self.patch_b,
             "encoder.embeddings.row_embedder.weight": self.row_emb,
             "encoder.embeddings.column_embedder.weight": self.col_emb,
             "encoder.layernorm.weight": self.enc_norm, "decoder.embed_tokens.weight": self.embed,
             "decoder.final_layer_norm.weight": self.dec_norm, "decoder.lm_head.weight": self.lm_head,
             "decoder.layer.0.self_attention.attention.relative_attention_bias.weight": self.rel_bias}
        inner = c.v_heads * c.v_dkv
        for i, L in enumerate(self.enc_layers):
            p = f"encoder.encoder.layer.{i}."
            for j, n in enumerate(("query", "key", "value")):
                w[p + f"attention.{n}.weight"] = L["wqkv"][j * inner:(j + 1) * inner]
            w.update({p + "attention.output.weight": L["wo"], p + "mlp.wi_0.weight": L["wi"][:c.v_ff],
                      p + "mlp.wi_1.weight": L["wi"][c.v_ff:], p + "mlp.wo.weight": L["wout"],
                      p + "pre_attention_layer_norm.weight": L["ln1"], p + "pre_mlp_layer_norm.weight": L["ln2"]})
        H = c.t_hidden
        for i, L in enumerate(self.dec_layers):
            p = f"decoder.layer.{i}."
            s, x = p + "self_attention.", p + "encoder_decoder_attention."
            for j, n in enumerate(("query", "key", "value")):
                w[s + f"attention.{n}.weight"] = L["wqkv"][j * H:(j + 1) * H]
            kv = self.w_xkv[2 * H * i: 2 * H * (i + 1)]
            w.update({s + "attention.output.weight": L["wo"], s + "layer_norm.weight": L["ln_s"],
                      x + "attention.query.weight": L["wq_x"], x + "attention.key.weight": kv[:H],
                      x + "attention.value.weight": kv[H:], x + "attention.output.weight": L["wo_x"],
                      x + "layer_norm.weight": L["ln_x"], p + "mlp.layer_norm.weight": L["ln_f"],
                      p + "mlp.DenseReluDense.wi_0.weight": L["wi"][:c.t_ff],
                      p + "mlp.DenseReluDense.wi_1.weight": L["wi"][c.t_ff:],
                      p + "mlp.DenseReluDense.wo.weight": L["wout"]})
        return w

    # -- encoder
    @torch.no_grad()
    def encode(self, patches: Sequence[torch.Tensor]) -> Tuple[torch.Tensor, torch.Tensor]:
        """Real patches of each image ([n_i, 2 + patch_dim], from :func:`flatten_patches`) ->
        (encoder rows packed [sum n_i, hidden], cu offsets int32 [B + 1])."""
        c, dev = self.cfg, self.device
        lens = [int(p.shape[0]) for p in patches]
        P = torch.cat(list(patches)).to(dev)
        rows, cols = P[:, 0].long(), P[:, 1].long()
        x = torch.addmm(self.patch_b, P[:, 2:].to(self.dtype), self.patch_w.t())
        x += self.row_emb.index_select(0, rows)
        x += self.col_emb.index_select(0, cols)
        cu = torch.tensor([0] + list(np.cumsum(lens)), dtype=torch.int32, device=dev)
        inner = c.v_heads * c.v_dkv
        h = ops.rmsnorm(x, self.enc_layers[0]["ln1"], c.eps)
        n = len(self.enc_layers)
        for li, L in enumerate(self.enc_layers):
            qkv = h @ L["wqkv"].t()
            a = ops.varlen_attention(qkv[:, :inner], qkv[:, inner:2 * inner], qkv[:, 2 * inner:], cu,
                                     c.v_heads, c.v_heads, c.v_dkv, max(lens), 1.0, causal=False)
            h = ops.add_rmsnorm(x, a @ L["wo"].t(), L["ln2"], c.eps)          # x += attention
            m = ops.gelu_tanh_mul(h @ L["wi"].t()) @ L["wout"].t()
            nxt = self.enc_layers[li + 1]["ln1"] if li + 1 < n else self.enc_norm
            h = ops.add_rmsnorm(x, m, nxt, c.eps)                               # x += MLP
        return h, cu

    # -- decoder
    def _bias_table(self, T: int) -> torch.Tensor:
        """[heads, T, T] fp32: relative position bias of query t over key j, -inf for j > t."""
        c = self.cfg
        pos = torch.arange(T, device=self.device)
        rel = pos[None, :] - pos[:, None]
        b = self.rel_bias[relative_bucket(rel, c.rel_buckets, c.rel_max_distance)]    # [T, T, heads]
        b = b.permute(2, 0, 1).contiguous()
        return b.masked_fill((rel > 0)[None], float("-inf"))

    def _cross_kv(self, enc: torch.Tensor, cu: torch.Tensor) -> dict:
        """Every layer's cross-attention K / V in the paged layout of the attention kernels
        (K pages [L, blocks, heads, 64, dkv], V^T pages [L, blocks, heads, dkv, 64]; image b
        owns blocks [b * nb, (b + 1) * nb)), computed by one GEMM over the encoder rows. The
        decoder's cross-attention is then the paged non-causal MFMA attention kernel with
        ``ctx_lens`` = each image's patch count (no mask tensor, padding never read)."""
        c, dev = self.cfg, enc.device
        lens = (cu[1:] - cu[:-1]).tolist()
        B, L, h, d = len(lens), c.t_layers, c.t_heads, c.t_dkv
        nb = -(-max(lens) // 64)
        kv = enc @ self.w_xkv.t()                                                   # [T, L*2H]
        pad = torch.zeros(B, nb * 64, kv.shape[1], dtype=kv.dtype, device=dev)
        for b, (s, n) in enumerate(zip(cu[:-1].tolist(), lens)):
            pad[b, :n] = kv[s:s + n]
        pad = pad.view(B, nb, 64, L, 2, h, d)
        kp = pad[:, :, :, :, 0].permute(3, 0, 1, 4, 2, 5).reshape(L, B * nb, h, 64, d).contiguous()
        vp = pad[:, :, :, :, 1].permute(3, 0, 1, 4, 5, 2).reshape(L, B * nb, h, d, 64).contiguous()
        return {"k": kp, "v": vp,
                "bt": torch.arange(B * nb, dtype=torch.int32, device=dev).view(B, nb),
                "lens": torch.tensor(lens, dtype=torch.int32, device=dev)}

    def _cross(self, q: torch.Tensor, xa: dict, li: int, T: int) -> torch.Tensor:
        """Cross-attention of q rows [B * T, H] (T decoder positions per image, image-major)."""
        c = self.cfg
        B = xa["lens"].numel()
        cu_q = xa.get(("cu_q", T))
        if cu_q is None:        # built once per decoder length (outside any graph replay)
            cu_q = xa[("cu_q", T)] = torch.arange(0, B * T + 1, T, dtype=torch.int32, device=q.device)
        return ops.prefill_attention_paged(q, xa["k"][li], xa["v"][li], xa["bt"], cu_q, xa["lens"],
                                           c.t_heads, c.t_heads, c.t_dkv, T, 1.0, causal=False)

    @staticmethod
    def _attend(q, k, v, bias):
        """Unscaled T5 attention softmax(q k^T + bias) v as one fused SDPA call (fp32 softmax
        inside; K / V are read once in their storage dtype, never widened in memory)."""
        return torch.nn.functional.scaled_dot_product_attention(q, k, v, attn_mask=bias, scale=1.0)

    def _dec_stack(self, x, B, T, bias, xa, kv_sink):
        """All decoder layers on the residual stream x [B*T, H] (updated in place) -> the
        final-normed rows. Per layer: one fused QKV GEMM; ``kv_sink(li, k, v)`` with this call's
        keys / values [B, heads, T, dkv] returns the (K, V) the self-attention reads (the
        teacher-forced path: these; the decode step: the cache they were written into); each
        residual add is fused into the following RMSNorm (``ops.add_rmsnorm``)."""
        c = self.cfg
        H, h, d = c.t_hidden, c.t_heads, c.t_dkv
        layers = self.dec_layers
        n = ops.rmsnorm(x, layers[0]["ln_s"], c.eps)
        for li, L in enumerate(layers):
            qkv = (n @ L["wqkv"].t()).view(B, T, 3, h, d)
            q = qkv[:, :, 0].transpose(1, 2)
            K, V = kv_sink(li, qkv[:, :, 1].transpose(1, 2), qkv[:, :, 2].transpose(1, 2))
            a = self._attend(q, K, V, bias).transpose(1, 2).reshape(B * T, H)
            n = ops.add_rmsnorm(x, a @ L["wo"].t(), L["ln_x"], c.eps)
            a = self._cross(n @ L["wq_x"].t(), xa, li, T)
            n = ops.add_rmsnorm(x, a @ L["wo_x"].t(), L["ln_f"], c.eps)
            m = ops.gelu_tanh_mul(n @ L["wi"].t()) @ L["wout"].t()
            nxt = layers[li + 1]["ln_s"] if li + 1 < len(layers) else self.dec_norm
            n = ops.add_rmsnorm(x, m, nxt, c.eps)
        return n

    @torch.no_grad()
    def decode_logits(self, enc: torch.Tensor, cu: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
        """Teacher-forced decoder: ids [B, T] -> logits [B, T, vocab] (fp32)."""
        B, T = ids.shape
        xa = self._cross_kv(enc, cu)
        bias = self._bias_table(T)[None].to(self.dtype)
        x = self.embed.index_select(0, ids.reshape(-1).to(self.device)).contiguous()
        y = self._dec_stack(x, B, T, bias, xa, lambda li, k, v: (k, v))
        return (y @ self.lm_head.t()).float().view(B, T, -1)

    # -- generation
    def _step(self, st: dict) -> None:
        """One greedy decode step on the static buffers of ``st`` (graph-capturable: the step
        index ``t`` is a device tensor; no host reads)."""
        c = self.cfg
        B = st["tok"].shape[0]
        t = st["t"]
        x = self.embed.index_select(0, st["tok"]).contiguous()
        bias = st["bias"].index_select(1, t).unsqueeze(0)                 # [1, heads, 1, S]

        def sink(li, k, v):                                               # k / v [B, heads, 1, dkv]
            st["k"][li].index_copy_(2, t, k)
            st["v"][li].index_copy_(2, t, v)
            return st["k"][li], st["v"][li]

        y = self._dec_stack(x, B, 1, bias, st["xa"], sink)
        logits = (y @ self.lm_head.t()).float()
        nxt = torch.argmax(logits, -1)
        # rows that already emitted EOS keep emitting padding
        nxt = torch.where(st["done"], torch.full_like(nxt, c.pad_id), nxt)
        if not st["ignore_eos"]:
            st["done"] |= nxt == c.eos_id
        st["tok"].copy_(nxt)
        st["out"].index_copy_(1, t, nxt.unsqueeze(1))
        t += 1

    @torch.no_grad()
    def generate(self, patches: Sequence[torch.Tensor], max_new_tokens: int = 512,
                 use_graph: Optional[bool] = None, ignore_eos: bool = False) -> List[List[int]]:
        """Greedy generation for a batch of images (their real patches). Returns each image's
        token ids up to (excluding) EOS. On a GPU the decode step replays as a hipGraph.
        ``ignore_eos``: every row runs all ``max_new_tokens`` steps (fixed-work benchmarks).
        Runs on request threads: the encoder, the warm-up step and the capture hold
        ``capture_guard`` (their library GEMMs never launch beside another thread's graph
        capture); graph replays do not, so a long generation never holds up an LLM engine
        that needs to capture a step graph meanwhile."""
        return self._generate(patches, max_new_tokens, use_graph, ignore_eos)

    def _generate(self, patches, max_new_tokens, use_graph, ignore_eos):
        c, dev = self.cfg, self.device
        if use_graph is None:
            use_graph = dev.type == "cuda"
        with capture_guard():
            st, graph = self._prepare(patches, max_new_tokens, use_graph, ignore_eos)
        S = int(max_new_tokens)
        for i in range(S):
            if graph is not None:
                graph.replay()
            else:
                with capture_guard():   # eager steps issue library GEMMs
                    self._step(st)
            if (i + 1) % 32 == 0 and bool(st["done"].all()):
                break
        out = st["out"].tolist()
        if ignore_eos:
            return out
        return [r[: r.index(c.eos_id)] if c.eos_id in r else r for r in out]

    def _prepare(self, patches, max_new_tokens, use_graph, ignore_eos):
        """Encoder pass, decode state and (use_graph) the captured decode step."""
        c, dev = self.cfg, self.device
        enc, cu = self.encode(patches)
        B, S = len(patches), int(max_new_tokens)
        st = {"xa": self._cross_kv(enc, cu), "bias": self._bias_table(S).to(self.dtype),
              "k": torch.zeros(c.t_layers, B, c.t_heads, S, c.t_dkv, dtype=self.dtype, device=dev),
              "v": torch.zeros(c.t_layers, B, c.t_heads, S, c.t_dkv, dtype=self.dtype, device=dev),
              "tok": torch.full((B,), c.decoder_start_id, dtype=torch.long, device=dev),
              "t": torch.zeros(1, dtype=torch.long, device=dev),
              "done": torch.zeros(B, dtype=torch.bool, device=dev),
              "out": torch.full((B, S), c.pad_id, dtype=torch.long, device=dev), "ignore_eos": ignore_eos}
        graph = None
        if use_graph:
            # warm up on a side stream (allocator pools, hipBLASLt handles), then capture one
            # step; the warm-up step is undone by resetting the state it advanced
            s = torch.cuda.Stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                self._step(st)
            torch.cuda.current_stream(dev).wait_stream(s)
            graph = torch.cuda.CUDAGraph()
            with capture_guard(), torch.cuda.graph(graph, stream=s, capture_error_mode="thread_local"):
                self._step(st)
            st["t"].zero_()
            st["done"].zero_()
            st["tok"].fill_(c.decoder_start_id)
            st["out"].fill_(c.pad_id)
        return st, graph


class DePlot:
    """Chart -> linearised data table (the reference's ``process_graph`` call). ``describe``
    takes image bytes and the prompt; in VQA mode the prompt is rendered as the header."""

    PROMPT = "Generate underlying data table of the figure below:"

    def __init__(self, cfg="deplot", device=None, weights=None, seed: int = 0, tokenizer=None):
        from ..utils.tokenizer import llm_tokenizer

        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        dtype = torch.bfloat16 if str(device).startswith("cuda") else torch.float32
        self.model = Pix2StructModel(cfg, device=device, dtype=dtype, weights=weights, seed=seed)
        self.cfg = self.model.cfg
        self.tok = tokenizer or llm_tokenizer()

    def patches(self, image, prompt: Optional[str] = None) -> torch.Tensor:
        """Header render on the host (PIL text), the per-pixel work on the model's device."""
        if self.cfg.is_vqa:
            image = render_header(image, prompt or self.PROMPT)
        return flatten_patches(image, self.cfg.max_patches, self.cfg.patch, device=self.model.device)

    def describe_batch(self, images: Sequence, prompt: Optional[str] = None,
                       max_new_tokens: int = 512) -> List[str]:
        ps = [self.patches(im, prompt) for im in images]
        outs = self.model.generate(ps, max_new_tokens=max_new_tokens)
        # the checkpoint's own tokenizer is not shipped here: ids fold into the framework
        # tokenizer's id space (``decode`` folds; random-init weights produce no real tables)
        return [self.tok.decode(o) for o in outs]

    def generate_many(self, images: Sequence, prompt: Optional[str] = None, batch: int = 32,
                      max_new_tokens: int = 512, threads: int = 8, ignore_eos: bool = False) -> List[List[int]]:
        """Token ids for many images in batches of ``batch``. The host part of the next batch
        (PNG decode + header render; PIL releases the GIL) runs on ``threads`` worker threads
        while the GPU encodes and decodes the current one; the per-pixel preprocessing runs on
        the device."""
        from concurrent.futures import ThreadPoolExecutor

        c = self.cfg
        prompt = prompt or self.PROMPT
        chunks = [list(images[i:i + batch]) for i in range(0, len(images), batch)]
        if not chunks:
            return []

        def host(im):
            return render_header(im, prompt) if c.is_vqa else _to_rgb_array(im)

        out: List[List[int]] = []
        with ThreadPoolExecutor(max(1, threads)) as pool:
            fut = [pool.submit(host, im) for im in chunks[0]]
            for i in range(len(chunks)):
                arrs = [f.result() for f in fut]
                if i + 1 < len(chunks):
                    fut = [pool.submit(host, im) for im in chunks[i + 1]]
                ps = [flatten_patches(a, c.max_patches, c.patch, device=self.model.device) for a in arrs]
                out += self.model.generate(ps, max_new_tokens=max_new_tokens, ignore_eos=ignore_eos)
        return out

    def describe(self, image, prompt: Optional[str] = None, max_new_tokens: int = 512) -> str:
        return self.describe_batch([image], prompt, max_new_tokens)[0]


class DePlotBatcher:
    """Dynamic batching for a served DePlot: chart requests arriving within ``max_delay_s`` of
    each other (up to ``max_batch`` images) share one encoder pass and one batched hipGraph
    decode; each request's tokens are cut at its own ``max_new_tokens``. Header rendering is
    per image, so requests with different prompts batch together."""

    def __init__(self, deplot: DePlot, max_batch: int = 32, max_delay_s: float = 0.02):
        import queue
        import threading

        self.dp, self.max_batch, self.max_delay_s = deplot, int(max_batch), float(max_delay_s)
        self.q = queue.Queue()
        self.batches = 0
        self._t = threading.Thread(target=self._run, daemon=True, name="deplot-batcher")
        self._t.start()

    def submit(self, image, prompt: Optional[str] = None, max_new_tokens: int = 512):
        from concurrent.futures import Future

        f = Future()
        self.q.put((image, prompt, int(max_new_tokens), f))
        return f

    def describe(self, image, prompt: Optional[str] = None, max_new_tokens: int = 512) -> str:
        return self.submit(image, prompt, max_new_tokens).result()

    def _run(self):
        import queue
        import time

        while True:
            items = [self.q.get()]
            deadline = time.monotonic() + self.max_delay_s
            while len(items) < self.max_batch:
                rem = deadline - time.monotonic()
                if rem <= 0:
                    break
                try:
                    items.append(self.q.get(timeout=rem))
                except queue.Empty:
                    break
            try:
                ps = [self.dp.patches(im, pr) for im, pr, _, _ in items]
                outs = self.dp.model.generate(ps, max_new_tokens=max(n for _, _, n, _ in items))
                self.batches += 1
                for (_, _, n, f), o in zip(items, outs):
                    f.set_result(self.dp.tok.decode(o[:n]))
            except Exception as e:  # noqa: BLE001 - delivered to every waiting request
                for *_, f in items:
                    if not f.done():
                        f.set_exception(e)
