"""Decoder-based cross-encoder reranker (NeMo Retriever's ``nv-rerank-qa-mistral-4b``, the
reference's ranking microservice: deploy/compose/docker-compose-nim-ms.yaml:58-84,
compose.env:31-33).

That model is Mistral-7B cut to its first 16 layers, run with a bidirectional attention mask,
mean-pooled over the pair's tokens and scored by a linear head; pairs are rendered as
``"question:{query} \\n \\n passage:{passage}"`` and capped at 512 tokens
(experimental/fm-asr-streaming-rag/nemo-retriever/model_configs/nv-rerank-qa-mistral-4b-A6000.yaml:1-16).

The forward reuses the decoder's weights and kernels over packed pairs with no KV cache:
RMSNorm (fused residual add), the fused QKV GEMM, RoPE without a cache write
(``ops.rope_cache_`` with no slots), packed *bidirectional* GQA MFMA attention
(``ops.varlen_attention(causal=False)``, head_dim 128), the SwiGLU MLP, then a masked mean
pool (``ops.pool_l2norm``) and the linear head. It plugs into :class:`EmbeddingEngine` (the
``/v1/ranking`` path) through the ``encoder=`` / ``encode_pair`` hooks.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch

from .. import ops
from .config import EncoderConfig, llama_config
from .llama import LlamaModel

RANKER_TEMPLATE = "question:{query} \n \n passage:{passage}"

# decoder preset + head size of each decoder ranker
DECODER_RANKERS = {
    "nv-rerank-qa-mistral-4b": "mistral-4b-rerank",
    "mistral-rerank-tiny": "mistral-tiny",
    "mistral-rerank-small": "mistral-small",
}


def ranker_encoder_config(name: str) -> EncoderConfig:
    """The EmbeddingEngine-facing config of a decoder ranker (hidden, 512-token window)."""
    d = llama_config(DECODER_RANKERS[name])
    return EncoderConfig(name=name, vocab_size=d.vocab_size, hidden=d.hidden, layers=d.layers,
                         heads=d.heads, ffn=d.ffn, max_position=512, pooling="mean",
                         normalize=False, query_prefix="", num_labels=1)


class DecoderRanker:
    def __init__(self, name: str = "nv-rerank-qa-mistral-4b", device="cuda", dtype=torch.bfloat16,
                 weights: Optional[Dict[str, torch.Tensor]] = None, seed: int = 0, max_len: int = 512):
        cfg = llama_config(DECODER_RANKERS[name])
        # bidirectional: no sliding window either (every pair fits the 512-token window)
        if weights is not None and "lm_head.weight" not in weights and not cfg.tie_embeddings:
            weights = {**weights, "lm_head.weight": weights["model.embed_tokens.weight"]}
        self.lm = LlamaModel(cfg, device, dtype=dtype, weights=weights, seed=seed)
        self.lm.lm_head = None                    # scoring head instead of the LM head
        self.cfg = cfg
        self.max_len = max_len
        dev = torch.device(device)
        if weights is not None and "score.weight" in weights:
            self.head_w = weights["score.weight"].to(dev, dtype)
            self.head_b = weights.get("score.bias", torch.zeros(1)).to(dev, torch.float32)
        else:
            g = torch.Generator(device=dev).manual_seed(seed + 5)
            self.head_w = torch.empty(1, cfg.hidden, device=dev, dtype=dtype).normal_(0, 0.02, generator=g)
            self.head_b = torch.zeros(1, device=dev, dtype=torch.float32)
        self._tok = None

    def state_dict(self) -> Dict[str, torch.Tensor]:
        """Decoder weights (HF names) plus the ``score`` head."""
        out = {k: v for k, v in self.lm.state_dict().items() if k != "lm_head.weight"}
        out["score.weight"] = self.head_w
        out["score.bias"] = self.head_b
        return out

    # ---------------------------------------------------------------- tokenisation
    @property
    def tok(self):
        if self._tok is None:
            from ..utils.tokenizer import llm_tokenizer

            self._tok = llm_tokenizer()
        return self._tok

    def encode_pair(self, query: str, passage: str, truncate: str = "END") -> List[int]:
        ids = [self.tok.bos_id] + self.tok.encode(RANKER_TEMPLATE.format(query=query, passage=passage))
        if len(ids) > self.max_len:
            if truncate == "NONE":
                raise ValueError(f"pair of {len(ids)} tokens exceeds {self.max_len} (truncate=NONE)")
            ids = ids[: self.max_len] if truncate != "START" else [ids[0]] + ids[-(self.max_len - 1):]
        V = self.cfg.vocab_size
        return [t % V for t in ids]

    # ---------------------------------------------------------------- forward
    @torch.inference_mode()
    def forward(self, ids: torch.Tensor, pos: torch.Tensor, cu: torch.Tensor, max_len: int,
                type_ids: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Packed pairs -> [B, 1] fp32 relevance logits."""
        h = packed_hidden(self.lm, ids, pos, cu, max_len, causal=False)
        pooled = ops.pool_l2norm(h, cu, 1, False)                     # masked mean, fp32
        return pooled @ self.head_w.float().t() + self.head_b


def packed_hidden(m: LlamaModel, ids: torch.Tensor, pos: torch.Tensor, cu: torch.Tensor, max_len: int,
                  causal: bool) -> torch.Tensor:
    """Final-normed hidden rows of packed sequences through a decoder's weights and kernels,
    with no KV cache: RMSNorm (fused residual add), the fused QKV GEMM, RoPE without a cache
    write, packed GQA MFMA attention (bidirectional for the ranker, causal for the reward
    model), the MLP."""
    hq, hkv, D = m.hq, m.hkv, m.D
    qd, kd = hq * D, hkv * D
    resid = m.embed_tokens(ids)
    L0 = m.layers[0]
    x = m._norm(resid, L0["attn_norm"], L0.get("attn_norm_b"))
    n = len(m.layers)
    d = None
    for li in range(n):
        L = m.layers[li]
        qkv = m._qkv(x, L)
        ops.rope_cache_(qkv, pos, m.cos_sin, None, None, None, hq, hkv, D)
        a = ops.varlen_attention(qkv[:, :qd], qkv[:, qd:qd + kd], qkv[:, qd + kd:], cu, hq, hkv, D,
                                 max_len, m.scale, causal=causal)
        o = m._bias_rank0(m._lin(a, L, "wo"), L.get("bo"))
        x = m._add_norm(resid, o, L["mlp_norm"], L.get("mlp_norm_b"))
        d = m._mlp(x, L)
        if li + 1 < n:
            Ln = m.layers[li + 1]
            x = m._add_norm(resid, d, Ln["attn_norm"], Ln.get("attn_norm_b"))
    return m._add_norm(resid, d, m.final_norm, m.final_norm_b)
