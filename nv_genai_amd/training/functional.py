"""Differentiable forwards for training.

The serving forwards (models/llama.py, models/encoder.py) run packed tokens through the
hand-written gfx950 kernels, which have no backward. Training runs the same weights through
autograd-capable PyTorch-ROCm ops on padded ``[B, S]`` batches:

* matmuls in bf16 (``torch.autocast``) on MFMA via hipBLASLt, fp32 accumulation;
* attention through ``F.scaled_dot_product_attention`` (the flash/memory-efficient backends
  of PyTorch-ROCm), causal for the LLM, key-padding-masked for the encoder;
* RMSNorm / LayerNorm / softmax statistics in fp32.

Parameters are taken from the serving model objects by reference (no copy), so a LoRA
adapter trained here merges straight back into a ``LlamaModel`` that the engine serves; full
fine-tuning keeps an fp32 master copy (``trainable_params``).

Reference behaviour: NeMo Megatron GPT SFT/LoRA (models/Gemma/lora.ipynb, sft.ipynb;
``peft_scheme=lora`` on ``attention_qkv``) and Megatron-SBERT fine-tuning
(experimental/synthetic-data-retriever-customization/retriever_customization.ipynb#cell 29).
"""
from __future__ import annotations

from typing import Callable, Dict, Optional

import torch
import torch.nn.functional as F
from torch.utils.checkpoint import checkpoint as _ckpt

LinearFn = Callable[[torch.Tensor, int, str], torch.Tensor]


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (y * w.float()).to(x.dtype)


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """Rotate-half RoPE. x [B, S, h, D]; cos/sin [B or 1, S, 1, D/2] fp32."""
    h = x.shape[-1] // 2
    x1, x2 = x[..., :h].float(), x[..., h:].float()
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1).to(x.dtype)


def _window_mask(S: int, W: int, device) -> torch.Tensor:
    """[S, S] bool: key j visible to query i iff i - W < j <= i."""
    i = torch.arange(S, device=device)
    d = i[:, None] - i[None, :]
    return (d >= 0) & (d < W)


def llama_hidden(model, ids: torch.Tensor, linear: Optional[LinearFn] = None,
                 params: Optional[Dict] = None, grad_ckpt: bool = False,
                 pos: Optional[torch.Tensor] = None) -> torch.Tensor:
    """ids [B, S] → final-normed hidden [B, S, H] (causal). ``linear(x, layer, name)``
    computes a projection (base weight + adapter); ``params`` overrides the model's tensors
    (fp32 masters for full fine-tuning).

    Every decoder family of ``LlamaConfig`` (the serving model's weights, same semantics as
    models/llama.py): LayerNorm + biases and the non-gated GELU MLP (StarCoder2), GeGLU and
    the scaled embedding (Gemma: its (1 + w) norm scale is already folded into the stored
    weight), sliding-window attention (Mistral v0.1, StarCoder2) and the sparse MoE MLP
    (Mixtral: dense per-expert loop over the routed rows, differentiable through the
    router's top-k weights)."""
    cfg = model.cfg
    P = params or {}
    B, S = ids.shape
    hq, hkv, D = model.hq, model.hkv, model.D
    if pos is None:
        pos = torch.arange(S, device=ids.device).unsqueeze(0).expand(B, S)
    cs = model.cos_sin.to(ids.device)[pos]                        # [B, S, D]
    cos, sin = cs[..., : D // 2].unsqueeze(2), cs[..., D // 2:].unsqueeze(2)
    dt = torch.bfloat16
    layer_norm = cfg.norm == "layer"
    amask = _window_mask(S, cfg.sliding_window, ids.device) if cfg.sliding_window and S > cfg.sliding_window else None

    def W(li, name):
        return P.get((li, name), model.layers[li].get(name) if li >= 0 else None)

    def lin(x, li, name, bias=None):
        y = linear(x, li, name) if linear is not None else x @ W(li, name).to(dt).t()
        b = W(li, bias) if bias else None
        return y if b is None else y + b.to(y.dtype)

    def norm(x, li, name):
        w = W(li, name) if li >= 0 else P.get(name, getattr(model, name))
        if not layer_norm:
            return rms_norm(x, w, cfg.eps)
        b = W(li, name + "_b") if li >= 0 else P.get(name + "_b", getattr(model, name + "_b"))
        return F.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), cfg.eps).to(x.dtype)

    def act(g):
        return F.silu(g) if cfg.act == "silu" else F.gelu(g, approximate="tanh")

    def mlp(h, li):
        if cfg.is_moe:
            x2 = h.reshape(-1, h.shape[-1])
            logits = (x2 @ W(li, "router").to(dt).t()).float()
            pr = torch.softmax(logits, -1)
            wk, ids_k = torch.topk(pr, cfg.experts_per_tok, -1)
            wk = wk / wk.sum(-1, keepdim=True)
            w13, w2 = W(li, "w13"), W(li, "w2")
            Fe = w2.shape[2]
            out = torch.zeros(x2.shape, dtype=torch.float32, device=x2.device)
            for e in range(w13.shape[0]):
                tok, slot = torch.where(ids_k == model.expert0 + e)
                if tok.numel() == 0:
                    continue
                gu = x2[tok] @ w13[e].to(dt).t()
                y = (act(gu[:, :Fe]) * gu[:, Fe:]) @ w2[e].to(dt).t()
                out = out.index_add(0, tok, y.float() * wk[tok, slot].unsqueeze(1))
            return out.to(h.dtype).view_as(h)
        gu = lin(h, li, "wgu", "bgu")
        if cfg.gated_mlp:
            g, u = gu.chunk(2, dim=-1)
            return lin(act(g) * u, li, "wd", "bd")
        return lin(act(gu), li, "wd", "bd")

    emb = P.get("embed", model.embed)
    x = F.embedding(ids, emb).to(dt)
    if cfg.embed_scale != 1.0:
        x = x * torch.tensor(cfg.embed_scale, dtype=dt)

    def layer(x, li):
        h = norm(x, li, "attn_norm")
        qkv = lin(h, li, "wqkv", "bqkv")
        q, k, v = qkv.split([hq * D, hkv * D, hkv * D], dim=-1)
        q = apply_rope(q.view(B, S, hq, D), cos, sin).transpose(1, 2)
        k = apply_rope(k.view(B, S, hkv, D), cos, sin).transpose(1, 2)
        v = v.view(B, S, hkv, D).transpose(1, 2)
        if amask is None:
            a = F.scaled_dot_product_attention(q, k, v, is_causal=True, scale=model.scale, enable_gqa=hq != hkv)
        else:
            a = F.scaled_dot_product_attention(q, k, v, attn_mask=amask, scale=model.scale, enable_gqa=hq != hkv)
        a = a.transpose(1, 2).reshape(B, S, hq * D)
        x = x + lin(a, li, "wo", "bo")
        return x + mlp(norm(x, li, "mlp_norm"), li)

    for li in range(len(model.layers)):
        if grad_ckpt and torch.is_grad_enabled():
            x = _ckpt(layer, x, li, use_reentrant=False)
        else:
            x = layer(x, li)
    return norm(x, -1, "final_norm")


def lm_loss(model, hidden: torch.Tensor, labels: torch.Tensor, params: Optional[Dict] = None,
            chunk: int = 2048) -> torch.Tensor:
    """Mean next-token cross entropy over positions with ``labels >= 0`` (labels are already
    shifted: labels[b, t] is the target for hidden[b, t]). The vocab projection is chunked
    over tokens so [tokens, 128256] fp32 logits never materialise at once."""
    P = params or {}
    head = P.get("lm_head", P.get("embed") if model.lm_head is model.embed else None)
    head = (head if head is not None else model.lm_head).to(torch.bfloat16)
    h = hidden.reshape(-1, hidden.shape[-1])
    y = labels.reshape(-1)
    keep = (y >= 0).nonzero().squeeze(1)
    h, y = h.index_select(0, keep), y.index_select(0, keep)
    total = h.new_zeros((), dtype=torch.float32)
    for s in range(0, h.shape[0], chunk):
        lg = (h[s:s + chunk] @ head.t()).float()
        total = total + F.cross_entropy(lg, y[s:s + chunk], reduction="sum")
    return total / max(1, y.numel())


def encoder_embed(model, ids: torch.Tensor, mask: torch.Tensor, params: Optional[Dict] = None,
                  grad_ckpt: bool = False) -> torch.Tensor:
    """ids/mask [B, S] (right padded) → pooled [B, H] fp32 (L2-normalised when configured)."""
    cfg = model.cfg
    P = params or {}
    B, S = ids.shape
    H, nh, hd = cfg.hidden, cfg.heads, cfg.head_dim
    dt = torch.bfloat16

    def g(li, name):
        return P.get((li, name), model.layers[li][name])

    pos = torch.arange(S, device=ids.device)
    e = (F.embedding(ids, P.get("word", model.word)).float() + P.get("pos", model.pos)[pos].float()
         + P.get("type", model.type)[0].float())
    x = F.layer_norm(e, (H,), P.get("emb_ln_g", model.emb_ln[0]).float(), P.get("emb_ln_b", model.emb_ln[1]).float(),
                     cfg.eps).to(dt)
    amask = mask.bool()[:, None, None, :]

    def layer(x, li):
        qkv = F.linear(x, g(li, "wqkv").to(dt), g(li, "bqkv").to(dt))
        q, k, v = (t.view(B, S, nh, hd).transpose(1, 2) for t in qkv.split(H, dim=-1))
        a = F.scaled_dot_product_attention(q, k, v, attn_mask=amask, scale=model.scale)
        a = a.transpose(1, 2).reshape(B, S, H)
        o = F.linear(a, g(li, "wo").to(dt), g(li, "bo").to(dt))
        x = F.layer_norm((x.float() + o.float()), (H,), g(li, "ln1_g").float(), g(li, "ln1_b").float(), cfg.eps).to(dt)
        h = F.gelu(F.linear(x, g(li, "wi").to(dt), g(li, "bi").to(dt)).float()).to(dt)
        o2 = F.linear(h, g(li, "wo2").to(dt), g(li, "bo2").to(dt))
        return F.layer_norm((x.float() + o2.float()), (H,), g(li, "ln2_g").float(), g(li, "ln2_b").float(),
                            cfg.eps).to(dt)

    for li in range(len(model.layers)):
        x = _ckpt(layer, x, li, use_reentrant=False) if grad_ckpt and torch.is_grad_enabled() else layer(x, li)
    xf = x.float()
    if cfg.pooling == "cls":
        pooled = xf[:, 0]
    else:
        m = mask.float().unsqueeze(-1)
        pooled = (xf * m).sum(1) / m.sum(1).clamp_min(1.0)
    if cfg.normalize:
        pooled = pooled / pooled.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    return pooled


def trainable_params(model, kind: str = "llama") -> Dict:
    """fp32 master copies of every weight (full fine-tuning), keyed like ``params``."""
    out: Dict = {}
    if kind == "llama":
        out["embed"], out["final_norm"] = model.embed, model.final_norm
        if getattr(model, "final_norm_b", None) is not None:
            out["final_norm_b"] = model.final_norm_b
        if model.lm_head is not model.embed:   # tied embeddings train through "embed"
            out["lm_head"] = model.lm_head
        for li, L in enumerate(model.layers):
            for n, t in L.items():
                out[(li, n)] = t
    else:
        out.update(word=model.word, pos=model.pos, type=model.type, emb_ln_g=model.emb_ln[0], emb_ln_b=model.emb_ln[1])
        for li, L in enumerate(model.layers):
            for n, t in L.items():
                out[(li, n)] = t
    return {k: v.detach().float().clone().requires_grad_(True) for k, v in out.items()}


def write_back(model, params: Dict, kind: str = "llama") -> None:
    """Copy fp32 masters back into the serving model's bf16 tensors (in place)."""
    with torch.no_grad():
        for k, v in params.items():
            if isinstance(k, tuple):
                model.layers[k[0]][k[1]].copy_(v)
            elif kind == "llama":
                getattr(model, k).copy_(v)
            elif k.startswith("emb_ln"):
                model.emb_ln[0 if k.endswith("g") else 1].copy_(v)
            else:
                getattr(model, k).copy_(v)
