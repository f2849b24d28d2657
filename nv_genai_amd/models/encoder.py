"""BERT-large-class bidirectional encoder: the embedding engine (SURVEY.md §2.B N2,
snowflake-arctic-embed-l / NV-Embed-QA shape) and, with a 1-logit head, the cross-encoder
reranker (N3).

Sequences are packed (varlen, cu_seqlens) so no padding token is ever computed — the
Triton MiniLM config of the reference pads every batch to 512
(experimental/streaming_ingest_rag/docker/extras/all-MiniLM-L6-v2_config.pbtxt:1-45).
Per layer (post-LN BERT):
    qkv = x @ Wqkv^T + b                      hipBLASLt (bias fused in addmm)
    a   = varlen MFMA attention, no mask      K10 (attention_prefill.hip, non-paged)
    x   = LN(a @ Wo^T + bo + x)               K11 (residual fused into the LN kernel)
    h   = gelu(x @ Wi^T + bi)                 K11 (bias+GELU kernel)
    x   = LN(h @ Wo2^T + bo2 + x)
then CLS / masked-mean pooling + L2 normalisation in one kernel (K12).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch

from .. import ops
from .config import EncoderConfig


class EncoderModel:
    def __init__(self, cfg: EncoderConfig, device="cuda", dtype=torch.bfloat16, seed: int = 0,
                 weights: Optional[Dict[str, torch.Tensor]] = None):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        if weights is None:
            self._random_init(seed)
        else:
            self._load(weights)

    def _random_init(self, seed: int):
        cfg, dev, dt = self.cfg, self.device, self.dtype
        g = torch.Generator(device=dev)
        g.manual_seed(seed + 17)
        H, F = cfg.hidden, cfg.ffn

        def rnd(*shape, std=0.02):
            t = torch.empty(*shape, device=dev, dtype=dt)
            t.normal_(0.0, std, generator=g)
            return t

        def zeros(*shape):
            return torch.zeros(*shape, device=dev, dtype=dt)

        def ones(*shape):
            return torch.ones(*shape, device=dev, dtype=dt)

        self.word = rnd(cfg.vocab_size, H)
        self.pos = rnd(cfg.max_position, H)
        self.type = rnd(cfg.type_vocab, H)
        self.emb_ln = (ones(H), zeros(H))
        self.layers: List[Dict[str, torch.Tensor]] = []
        for _ in range(cfg.layers):
            self.layers.append({
                "wqkv": rnd(3 * H, H), "bqkv": zeros(3 * H),
                "wo": rnd(H, H), "bo": zeros(H), "ln1_g": ones(H), "ln1_b": zeros(H),
                "wi": rnd(F, H), "bi": zeros(F),
                "wo2": rnd(H, F), "bo2": zeros(H), "ln2_g": ones(H), "ln2_b": zeros(H),
            })
        if cfg.num_labels:
            self.cls_w = rnd(cfg.num_labels, H)
            self.cls_b = zeros(cfg.num_labels)

    def _load(self, w: Dict[str, torch.Tensor]):
        """HF BERT naming (embeddings.*, encoder.layer.N.*), prefix ``bert.`` optional."""
        dev, dt = self.device, self.dtype
        pre = "bert." if any(k.startswith("bert.") for k in w) else ""

        def get(n):
            return w[pre + n].to(dev, dt)

        self.word = get("embeddings.word_embeddings.weight")
        self.pos = get("embeddings.position_embeddings.weight")
        self.type = get("embeddings.token_type_embeddings.weight")
        self.emb_ln = (get("embeddings.LayerNorm.weight"), get("embeddings.LayerNorm.bias"))
        self.layers = []
        for i in range(self.cfg.layers):
            p = f"encoder.layer.{i}."
            q, k, v = (get(p + f"attention.self.{n}.weight") for n in ("query", "key", "value"))
            bq, bk, bv = (get(p + f"attention.self.{n}.bias") for n in ("query", "key", "value"))
            self.layers.append({
                "wqkv": torch.cat([q, k, v]).contiguous(), "bqkv": torch.cat([bq, bk, bv]),
                "wo": get(p + "attention.output.dense.weight"), "bo": get(p + "attention.output.dense.bias"),
                "ln1_g": get(p + "attention.output.LayerNorm.weight"), "ln1_b": get(p + "attention.output.LayerNorm.bias"),
                "wi": get(p + "intermediate.dense.weight"), "bi": get(p + "intermediate.dense.bias"),
                "wo2": get(p + "output.dense.weight"), "bo2": get(p + "output.dense.bias"),
                "ln2_g": get(p + "output.LayerNorm.weight"), "ln2_b": get(p + "output.LayerNorm.bias"),
            })
        if self.cfg.num_labels:
            self.cls_w = w["classifier.weight"].to(dev, dt)
            self.cls_b = w["classifier.bias"].to(dev, dt)

    def state_dict(self) -> Dict[str, torch.Tensor]:
        H = self.cfg.hidden
        out = {"embeddings.word_embeddings.weight": self.word,
               "embeddings.position_embeddings.weight": self.pos,
               "embeddings.token_type_embeddings.weight": self.type,
               "embeddings.LayerNorm.weight": self.emb_ln[0],
               "embeddings.LayerNorm.bias": self.emb_ln[1]}
        for i, L in enumerate(self.layers):
            p = f"encoder.layer.{i}."
            for j, n in enumerate(("query", "key", "value")):
                out[p + f"attention.self.{n}.weight"] = L["wqkv"][j * H:(j + 1) * H]
                out[p + f"attention.self.{n}.bias"] = L["bqkv"][j * H:(j + 1) * H]
            out[p + "attention.output.dense.weight"] = L["wo"]
            out[p + "attention.output.dense.bias"] = L["bo"]
            out[p + "attention.output.LayerNorm.weight"] = L["ln1_g"]
            out[p + "attention.output.LayerNorm.bias"] = L["ln1_b"]
            out[p + "intermediate.dense.weight"] = L["wi"]
            out[p + "intermediate.dense.bias"] = L["bi"]
            out[p + "output.dense.weight"] = L["wo2"]
            out[p + "output.dense.bias"] = L["bo2"]
            out[p + "output.LayerNorm.weight"] = L["ln2_g"]
            out[p + "output.LayerNorm.bias"] = L["ln2_b"]
        if self.cfg.num_labels:
            out["classifier.weight"] = self.cls_w
            out["classifier.bias"] = self.cls_b
        return out

    def forward(self, ids: torch.Tensor, pos: torch.Tensor, cu: torch.Tensor, max_len: int,
                type_ids: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Packed tokens -> pooled [B, H] fp32 (L2-normalised unless configured otherwise);
        for a reranker (num_labels > 0) returns [B, num_labels] fp32 logits."""
        cfg = self.cfg
        H, nh, hd = cfg.hidden, cfg.heads, cfg.head_dim
        tt = self.type[0] if type_ids is None else None
        e = torch.nn.functional.embedding(ids.long(), self.word)
        e = e + torch.nn.functional.embedding(pos.long(), self.pos)
        if type_ids is None:
            e = e + tt
        else:
            e = e + torch.nn.functional.embedding(type_ids.long(), self.type)
        x = ops.layernorm(e.contiguous(), self.emb_ln[0], self.emb_ln[1], cfg.eps)
        for L in self.layers:
            qkv = torch.addmm(L["bqkv"], x, L["wqkv"].t())
            a = ops.varlen_attention(qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:], cu, nh, nh, hd,
                                     max_len, self.scale, causal=False)
            o = torch.addmm(L["bo"], a, L["wo"].t())
            x = ops.layernorm(o, L["ln1_g"], L["ln1_b"], cfg.eps, resid=x)
            h = x @ L["wi"].t()
            ops.bias_gelu_(h, L["bi"])
            o2 = torch.addmm(L["bo2"], h, L["wo2"].t())
            x = ops.layernorm(o2, L["ln2_g"], L["ln2_b"], cfg.eps, resid=x)
        mode = 0 if cfg.pooling == "cls" else 1
        if cfg.num_labels:
            pooled = ops.pool_l2norm(x, cu, mode, False)
            return pooled @ self.cls_w.float().t() + self.cls_b.float()
        return ops.pool_l2norm(x, cu, mode, cfg.normalize)
