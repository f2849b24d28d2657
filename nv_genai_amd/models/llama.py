"""Decoder-only LMs (Llama-3 8B / 70B, Mistral, Mixtral MoE, Gemma, StarCoder2) on the
gfx950 kernel set, tensor-parallel over RCCL.

This is the MI355X-native replacement for the TensorRT-LLM engine inside NIM
(SURVEY.md §2.B N1). Per layer (Llama form; the other families switch pieces through
``LlamaConfig.arch`` flags, see :class:`nv_genai_amd.models.config.LlamaConfig`):

    x_norm = rmsnorm(resid)                          K3  (fused with the residual add)
    qkv    = x_norm @ Wqkv^T                         K6  hipBLASLt (column-parallel)
    rope + paged K/V^T cache write                   K4 + K9 (one kernel)
    attn   = prefill (MFMA flash, paged) | decode (MFMA paged GQA, split-K)   K1 / K2
    resid += all_reduce(attn @ Wo^T)                 K6 row-parallel + CC1
    x_norm = rmsnorm(resid)
    h      = silu(x_norm @ Wg^T) * (x_norm @ Wu^T)   K6 (fused gate|up GEMM) + K5
    resid += all_reduce(h @ Wd^T)                    K6 row-parallel + CC2

Only the rows that produce a token (the last prompt position of each sequence, every decode
row) go through the final norm and the vocab-parallel LM head (+ all-gather, CC4).

Family switches: LayerNorm+bias instead of RMSNorm (StarCoder2), biased projections
(hipBLASLt bias epilogue through ``torch.addmm``; row-parallel biases added on TP rank 0
only), GeGLU / non-gated GELU MLPs (``ops.gelu_tanh_mul`` / ``ops.bias_gelu_``), Gemma's
(1 + w) norm scale (folded into the stored weight) and sqrt(hidden) embedding scale, tied
embeddings, sliding-window attention (a kernel argument: pages older than the window are
never read), head_dim 256, and the sparse MoE MLP of Mixtral (``ops.moe_ffn``: routing,
gathered grouped MFMA GEMMs with a fused SwiGLU epilogue, weighted combine). Under TP the
experts are partitioned over the ranks (expert parallelism) when their count divides the
group, otherwise every expert's FFN is split like a dense MLP; either way the MoE output is
a partial sum that joins the dense path's all-reduce.
"""
from __future__ import annotations

import contextlib
import math
import os
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

from .. import ops
from ..ops import reference as ref
from ..parallel.comm import custom_all_reduce_for
from ..parallel.dist import (ParallelContext, get_context, tp_all_gather, tp_all_gather_rows,
                             tp_all_reduce, tp_reduce_scatter_rows)
from .config import LlamaConfig


@dataclass
class AttnMeta:
    """Per-step attention/cache layout (built by the engine from the native scheduler)."""

    kind: str                      # "prefill" | "decode"
    slots: torch.Tensor            # [T] int32 cache slot of each token (-1 = no write)
    cu_q: torch.Tensor             # [B+1] int32
    ctx_lens: torch.Tensor         # [B] int32 keys visible to each sequence
    block_tables: torch.Tensor     # [B, max_blocks] int32
    max_q_len: int
    max_ctx: int
    decode_ws: Optional[ops.DecodeWorkspace] = None
    n_decode: int = 0                          # mixed steps: rows [0, n_decode) are decode rows
    cu_q_prefill: Optional[torch.Tensor] = None  # mixed steps: cu_seqlens of the prefill rows
    # kind "graph" (a hipGraph-captured prefill / mixed step over a bucket of rows; every
    # step-dependent quantity lives in device buffers): decode rows [0, n_decode) read
    # decode_ctx (0 past the step's real decode rows: skipped), the prefill rows are covered
    # by the work list (items [k, 2], n_items [1]) over absolute token rows (cu_q / ctx_lens
    # of all the step's sequences); launch shape of the work-list kernel: (grid, ks)
    decode_ctx: Optional[torch.Tensor] = None
    items: Optional[torch.Tensor] = None
    n_items: Optional[torch.Tensor] = None
    pf_grid: int = 512
    pf_ks: int = 1
    pf_impl: int = 2    # 2: 32x32 kernel (bf16 head_dim-128 pages), 1: 16x16 kernel
    pf_seq: bool = False  # the work list after the decode attention on the main stream


class LlamaModel:
    """Decoder LM (every family of :class:`LlamaConfig`); ``DecoderModel`` is an alias."""

    def __init__(self, cfg: LlamaConfig, device="cuda", dtype=torch.bfloat16,
                 pctx: Optional[ParallelContext] = None, seed: int = 0,
                 weights: Optional[Dict[str, torch.Tensor]] = None, fp8: bool = False):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.kv_dtype, self.kv_scales = "auto", (1.0, 1.0)   # set by allocate_kv_cache
        self.p = pctx or get_context()
        tp = self.p.tp_size
        # expert parallelism: each TP rank owns num_experts / tp whole experts when that
        # divides; otherwise every expert's FFN is sharded like a dense MLP
        self.expert_parallel = cfg.is_moe and tp > 1 and cfg.num_experts % tp == 0
        ffn_tp = 1 if self.expert_parallel else tp
        # KV heads: split over the ranks, or — with more ranks than KV heads (Gemma-2B's one
        # KV head at TP=2, Llama-3-70B at TP=16) — replicated: each group of tp / kv_heads
        # ranks holds one KV head, exactly the one its query heads attend to
        kv_ok = cfg.kv_heads % tp == 0 or tp % cfg.kv_heads == 0
        if cfg.heads % tp or not kv_ok or cfg.ffn % ffn_tp or cfg.vocab_size % tp:
            raise ValueError(f"{cfg.name}: dims not divisible by tp={tp}")
        self.hq = cfg.heads // tp
        self.hkv = max(1, cfg.kv_heads // tp)
        self.kv_replicas = max(1, tp // cfg.kv_heads)
        self.D = cfg.head_dim
        self.ffn = cfg.ffn // ffn_tp
        self.n_experts = (cfg.num_experts // tp if self.expert_parallel else cfg.num_experts)
        self.expert0 = self.p.tp_rank * self.n_experts if self.expert_parallel else 0
        self.moe_ws = None    # ops.MoEWorkspace owned by the serving engine (GPU MoE)
        self.window = int(cfg.sliding_window or 0)
        self.vocab_local = cfg.vocab_size // tp
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        # pipeline stage: a contiguous slice of layers; stage 0 also holds the embedding and
        # the LM head (it samples), the last stage applies the final norm
        pp, s = self.p.pp_size, self.p.pp_rank
        if cfg.layers < pp:
            raise ValueError(f"{cfg.name}: {cfg.layers} layers cannot fill {pp} pipeline stages")
        self.layer_lo = s * cfg.layers // pp
        self.layer_hi = (s + 1) * cfg.layers // pp
        self.first_stage = s == 0
        self.last_stage = s == pp - 1
        if weights is None:
            self._random_init(seed)
        else:
            self._load(weights)
        self.cos_sin = ops.rope_cos_sin(cfg.max_position, cfg.head_dim, cfg.rope_theta,
                                        cfg.rope_scaling).to(self.device)
        self.split_mixed = False   # mixed steps on two streams (forward_split)
        # mixed steps: prefill attention on a side stream, concurrent with the decode
        # attention (HBM-bound, spare MFMA issue slots) on the main stream
        self.concurrent_attention = os.environ.get("NGA_CONCURRENT_ATTN", "1") != "0"
        self._attn_stream = None
        self._aux = None
        # sequence parallelism for TP prefill: norms and residual on T / tp rows, reduce-
        # scatter + all-gather instead of all-reduce (SURVEY.md §2.E "SP", §5.7)
        self.sequence_parallel = False
        self.sp_min_tokens = 512
        self.sp_steps = 0
        # o / down / gate-up projections of steps above 4,096 rows at hidden 4,096 (prefill
        # chunks or budgets past 4,096 tokens; the headline's steps stop at 4,096): the GEMM
        # rows cut at the last multiple of 4,096 — at M = 4,352 o 134.8 -> 119.6 us, down
        # 428 -> 373 us, gate/up 694 -> 686 us per layer (profiles/r3_rowsplit). q/k/v loses
        # (167 -> 184 us) and stays whole. NGA_ROW_SPLIT=0 turns it off
        self.row_split = os.environ.get("NGA_ROW_SPLIT", "1") != "0"
        # decode-shape projections (M <= 512 rows) on the skinny MFMA GEMM where the measured
        # table (ops.skinny) says it beats the library GEMM: K-split o / down partials summed by
        # the residual add + RMSNorm kernel, SwiGLU fused into gate / up, fp32 logits straight
        # from the LM head. One pipeline stage; under TP the table holds each rank's shard shapes
        # (llama3-70b TP=8) and row-parallel K-split partials are summed before the all-reduce
        # (``_reduce_add_norm``), so partial sums never cross a collective
        self.skinny = (self.device.type == "cuda" and dtype == torch.bfloat16
                       and self.p.pp_size == 1 and ops.skinny.enabled())
        self.fp8 = False
        if fp8:
            self.quantize_fp8()

    # ------------------------------------------------------------------ FP8 (W8A8)
    _LINEARS = ("wqkv", "wo", "wgu", "wd")

    def quantize_fp8(self) -> None:
        """W8A8 serving mode (the engine's int8/fp8 precision knob, TRT-LLM
        ``mistral-7b.yaml:34-35``; here OCP e4m3fn, gfx950's native FP8): the four projection
        weights of every layer become FP8 with one scale per output channel and the bf16 copies
        are freed; activations are quantised per token row by ``ops.quant_fp8_rows`` and the
        GEMMs run as row-scaled hipBLASLt FP8 GEMMs. Embedding, LM head, norms, attention and
        the KV cache stay bf16."""
        if self.fp8:
            return
        if self.cfg.is_moe or not self.cfg.gated_mlp or self.cfg.attn_bias or self.cfg.mlp_bias:
            raise NotImplementedError(f"FP8 W8A8 mode covers bias-free gated dense decoders, not {self.cfg.arch}")
        for L in self.layers:
            for n in self._LINEARS:
                L[n + "8"], L[n + "_s"] = ops.quantize_weight_fp8(L.pop(n))
        self.fp8 = True
        if self.device.type == "cuda":
            torch.cuda.empty_cache()

    def _pick(self, w: torch.Tensor, M: int):
        """(cfg, split) of the skinny GEMM for x[M, K] @ w^T, or None (library GEMM)."""
        if not self.skinny or self.fp8:
            return None
        return ops.skinny.table().pick(w.shape[0], w.shape[1], M)

    def _lin(self, x: torch.Tensor, L: dict, name: str, swiglu: bool = False, partial_ok: bool = False):
        """x @ W^T for projection ``name`` (bf16, or FP8 W8A8 when quantised); ``swiglu``:
        x is the [M, 2F] gate|up output and the projection consumes silu(gate) * up.
        ``partial_ok``: the caller sums K-split partials itself (``_reduce_add_norm``), so a
        skinny K-split result may come back as an ``ops.PartialSum``."""
        if not self.fp8:
            a = ops.silu_mul(x) if swiglu else x
            w = L[name]
            M = a.shape[0]
            if M == 1 and self.skinny and self._gemv_ok(a, w):
                # one row (batch-1 decode): the weight-streaming GEMV (profiles/r4_gemv/)
                return ops.gemv(a, w, 0)
            pk = self._pick(w, M)
            if pk is not None:
                cfg, split = pk
                if split == 1:
                    return ops.skinny_gemm(a, w, cfg, 1, 0)
                part = ops.PartialSum(ops.skinny_gemm(a, w, cfg, split, 1))
                return part if partial_ok else part.materialize()
            if self.row_split and name in ("wo", "wd", "wgu") and self.cfg.hidden == 4096 and M > 4096 and M % 4096:
                return ops.linear_rows_split(a, w, split=M // 4096 * 4096)
            return ops.linear(a, w)
        x8, sx = ops.quant_fp8_rows(x, mode=1 if swiglu else 0)
        return ops.fp8_linear(x8, sx, L[name + "8"], L[name + "_s"], x.shape[0])

    # ------------------------------------------------------------------ weights
    def _random_init(self, seed: int):
        cfg, dev, dt = self.cfg, self.device, self.dtype
        g = torch.Generator(device=dev)
        H = cfg.hidden
        staged = self.p.pp_size > 1

        def reseed(part: int):
            # pipeline stages: per-part seeds, so a layer's weights do not depend on which
            # stage builds it. One stage: one sequential stream (the weights every earlier
            # measurement in profiles/ used)
            if staged:
                g.manual_seed(seed * 1_000_003 + self.p.tp_rank * 10_007 + part)

        def rnd(*shape, std=0.02):
            t = torch.empty(*shape, device=dev, dtype=dt)
            t.normal_(0.0, std, generator=g)
            return t

        def ones(n):
            return torch.ones(n, device=dev, dtype=dt)

        def zeros(n):
            return torch.zeros(n, device=dev, dtype=dt)

        g.manual_seed(seed * 1000 + self.p.tp_rank)
        out_std = 0.02 / math.sqrt(2 * cfg.layers)
        reseed(0)
        self.embed = rnd(self.vocab_local, H) if self.first_stage else None
        self.layers: List[Dict[str, torch.Tensor]] = []
        qkv_rows = (self.hq + 2 * self.hkv) * self.D
        for i in range(self.layer_lo, self.layer_hi):
            reseed(i + 2)
            L = {
                "attn_norm": ones(H),
                "wqkv": rnd(qkv_rows, H),
                "wo": rnd(H, self.hq * self.D, std=out_std),
                "mlp_norm": ones(H),
            }
            if cfg.is_moe:
                E, F = self.n_experts, self.ffn
                L["router"] = rnd(cfg.num_experts, H)
                L["w13"] = rnd(E, 2 * F, H)
                L["w2"] = rnd(E, H, F, std=out_std)
            else:
                L["wgu"] = rnd((2 if cfg.gated_mlp else 1) * self.ffn, H)
                L["wd"] = rnd(H, self.ffn, std=out_std)
            if cfg.norm == "layer":
                L["attn_norm_b"], L["mlp_norm_b"] = zeros(H), zeros(H)
            if cfg.attn_bias:
                L["bqkv"], L["bo"] = zeros(qkv_rows), zeros(H)
            if cfg.mlp_bias:
                L["bgu"] = zeros((2 if cfg.gated_mlp else 1) * self.ffn)
                L["bd"] = zeros(H)
            self.layers.append(L)
        self.final_norm = ones(H)
        self.final_norm_b = zeros(H) if cfg.norm == "layer" else None
        reseed(1)
        if not self.first_stage:
            self.lm_head = None
        elif cfg.tie_embeddings:
            self.lm_head = self.embed
        else:
            self.lm_head = rnd(self.vocab_local, H)

    def _load(self, w: Dict[str, torch.Tensor]):
        """Load HF-named decoder weights (model.layers.N.self_attn.q_proj.weight, ...) of any
        supported family, fusing q/k/v (and gate/up), folding Gemma's (1 + w) norm scale, and
        slicing this rank's TP shard (experts: this rank's experts under expert parallelism)."""
        cfg, dev, dt = self.cfg, self.device, self.dtype
        tp, r = self.p.tp_size, self.p.tp_rank
        gemma = cfg.arch == "gemma"

        def rows(t, n=0):  # column-parallel shard (output rows)
            c = t.shape[0] // tp
            return t[r * c:(r + 1) * c]

        def cols(t):  # row-parallel shard (input columns)
            c = t.shape[1] // tp
            return t[:, r * c:(r + 1) * c]

        def kv_rows(t):  # K / V projection rows: this rank's KV heads (split or replicated)
            if self.kv_replicas == 1:
                return rows(t)
            h = r // self.kv_replicas
            return t[h * cfg.head_dim:(h + 1) * cfg.head_dim]

        def get(name):
            return w[name].to(dev, dt)

        def norm(name):
            t = get(name)
            return (t.float() + 1.0).to(dt) if gemma else t

        self.embed = rows(get("model.embed_tokens.weight")).contiguous() if self.first_stage else None
        self.layers = []
        for i in range(self.layer_lo, self.layer_hi):
            p = f"model.layers.{i}."
            a = p + "self_attn."
            q, k, v = get(a + "q_proj.weight"), get(a + "k_proj.weight"), get(a + "v_proj.weight")
            L = {
                "attn_norm": norm(p + "input_layernorm.weight"),
                "wqkv": torch.cat([rows(q), kv_rows(k), kv_rows(v)]).contiguous(),
                "wo": cols(get(a + "o_proj.weight")).contiguous(),
                "mlp_norm": norm(p + "post_attention_layernorm.weight"),
            }
            if cfg.norm == "layer":
                L["attn_norm_b"] = get(p + "input_layernorm.bias")
                L["mlp_norm_b"] = get(p + "post_attention_layernorm.bias")
            if cfg.attn_bias:
                L["bqkv"] = torch.cat([rows(get(a + "q_proj.bias")), kv_rows(get(a + "k_proj.bias")),
                                       kv_rows(get(a + "v_proj.bias"))]).contiguous()
                L["bo"] = get(a + "o_proj.bias")
            if cfg.is_moe:
                L.update(self._load_experts(w, p, get, rows))
            elif cfg.gated_mlp:
                gt, up = get(p + "mlp.gate_proj.weight"), get(p + "mlp.up_proj.weight")
                L["wgu"] = torch.cat([rows(gt), rows(up)]).contiguous()
                L["wd"] = cols(get(p + "mlp.down_proj.weight")).contiguous()
            else:   # StarCoder2: c_fc -> gelu -> c_proj
                L["wgu"] = rows(get(p + "mlp.c_fc.weight")).contiguous()
                L["wd"] = cols(get(p + "mlp.c_proj.weight")).contiguous()
                if cfg.mlp_bias:
                    L["bgu"] = rows(get(p + "mlp.c_fc.bias")).contiguous()
                    L["bd"] = get(p + "mlp.c_proj.bias")
            self.layers.append(L)
        self.final_norm = norm("model.norm.weight")
        self.final_norm_b = get("model.norm.bias") if cfg.norm == "layer" else None
        self.lm_head = None
        if self.first_stage:
            if cfg.tie_embeddings or "lm_head.weight" not in w:
                self.lm_head = self.embed
            else:
                self.lm_head = rows(get("lm_head.weight")).contiguous()

    def _load_experts(self, w, p, get, rows):
        """Mixtral experts in either checkpoint form: per-expert ``block_sparse_moe.experts.E.
        w1/w3/w2`` (the released checkpoints) or the fused ``mlp.experts.gate_up_proj`` /
        ``down_proj`` tensors of current transformers."""
        cfg = self.cfg
        ep = self.expert_parallel
        tp, r = self.p.tp_size, self.p.tp_rank
        E0, E = self.expert0, self.n_experts
        F = self.ffn

        def fsplit(t, dim):   # expert-TP: this rank's slice of the FFN dim
            if ep or tp == 1:
                return t
            return t.narrow(dim, r * F, F)

        if p + "mlp.experts.gate_up_proj" in w:
            gu = get(p + "mlp.experts.gate_up_proj")[E0:E0 + E]        # [E, 2F_full, H]
            Ff = gu.shape[1] // 2
            w13 = torch.cat([fsplit(gu[:, :Ff], 1), fsplit(gu[:, Ff:], 1)], 1)
            w2 = fsplit(get(p + "mlp.experts.down_proj")[E0:E0 + E], 2)
            router = get(p + "mlp.gate.weight")
        else:
            b = p + "block_sparse_moe."
            w13 = torch.stack([torch.cat([fsplit(get(b + f"experts.{e}.w1.weight"), 0),
                                          fsplit(get(b + f"experts.{e}.w3.weight"), 0)])
                               for e in range(E0, E0 + E)])
            w2 = torch.stack([fsplit(get(b + f"experts.{e}.w2.weight"), 1) for e in range(E0, E0 + E)])
            router = get(b + "gate.weight")
        assert router.shape[0] == cfg.num_experts
        return {"router": router.contiguous(), "w13": w13.contiguous(), "w2": w2.contiguous()}

    def state_dict(self) -> Dict[str, torch.Tensor]:
        """HF-named weights of this rank (unfused; TP shards are local slices; a pipeline
        stage holds only its layers, plus embedding and LM head on stage 0)."""
        if self.fp8:
            raise RuntimeError("state_dict of an FP8-quantised model: export the bf16 model before quantize_fp8()")
        cfg = self.cfg
        gemma = cfg.arch == "gemma"

        def unnorm(t):
            return (t.float() - 1.0).to(t.dtype) if gemma else t

        out = {"model.norm.weight": unnorm(self.final_norm)}
        if self.final_norm_b is not None:
            out["model.norm.bias"] = self.final_norm_b
        if self.first_stage:
            out["model.embed_tokens.weight"] = self.embed
            if not cfg.tie_embeddings:
                out["lm_head.weight"] = self.lm_head
        qd, kd = self.hq * self.D, self.hkv * self.D
        for i, L in enumerate(self.layers, start=self.layer_lo):
            p = f"model.layers.{i}."
            a = p + "self_attn."
            out[p + "input_layernorm.weight"] = unnorm(L["attn_norm"])
            out[a + "q_proj.weight"] = L["wqkv"][:qd]
            out[a + "k_proj.weight"] = L["wqkv"][qd:qd + kd]
            out[a + "v_proj.weight"] = L["wqkv"][qd + kd:]
            out[a + "o_proj.weight"] = L["wo"]
            out[p + "post_attention_layernorm.weight"] = unnorm(L["mlp_norm"])
            if "attn_norm_b" in L:
                out[p + "input_layernorm.bias"] = L["attn_norm_b"]
                out[p + "post_attention_layernorm.bias"] = L["mlp_norm_b"]
            if "bqkv" in L:
                out[a + "q_proj.bias"] = L["bqkv"][:qd]
                out[a + "k_proj.bias"] = L["bqkv"][qd:qd + kd]
                out[a + "v_proj.bias"] = L["bqkv"][qd + kd:]
                out[a + "o_proj.bias"] = L["bo"]
            if cfg.is_moe:
                out[p + "mlp.gate.weight"] = L["router"]
                out[p + "mlp.experts.gate_up_proj"] = L["w13"]
                out[p + "mlp.experts.down_proj"] = L["w2"]
            elif cfg.gated_mlp:
                out[p + "mlp.gate_proj.weight"] = L["wgu"][: self.ffn]
                out[p + "mlp.up_proj.weight"] = L["wgu"][self.ffn:]
                out[p + "mlp.down_proj.weight"] = L["wd"]
            else:
                out[p + "mlp.c_fc.weight"] = L["wgu"]
                out[p + "mlp.c_proj.weight"] = L["wd"]
                if "bgu" in L:
                    out[p + "mlp.c_fc.bias"] = L["bgu"]
                    out[p + "mlp.c_proj.bias"] = L["bd"]
        return out

    # ------------------------------------------------------------------ cache
    def allocate_kv_cache(self, num_blocks: int, block_size: int = 64, kv_dtype: str = "auto",
                          kv_scales=(1.0, 1.0)):
        """Paged K [layers, blocks, Hkv, 64, D] and Vᵀ [layers, blocks, Hkv, D, 64] caches.
        ``kv_dtype``: "auto" (the model dtype) or "fp8" — OCP e4m3fn pages holding k / k_scale
        and v / v_scale (half the bytes: twice the cached tokens, half the decode KV stream;
        the attention kernels widen the pages to bf16 in registers and fold the scales in)."""
        if block_size != 64:
            raise ValueError("the gfx950 attention kernels use 64-token KV pages")
        if kv_dtype not in ("auto", "bf16", "fp8"):
            raise ValueError(f"kv_dtype must be auto, bf16 or fp8, not {kv_dtype!r}")
        shape_k = (len(self.layers), num_blocks, self.hkv, block_size, self.D)
        shape_v = (len(self.layers), num_blocks, self.hkv, self.D, block_size)
        self.kv_dtype = kv_dtype if kv_dtype == "fp8" else "auto"
        self.kv_scales = (float(kv_scales[0]), float(kv_scales[1])) if kv_dtype == "fp8" else (1.0, 1.0)
        # zero-filled: masked keys of a partially filled page must stay finite
        if kv_dtype == "fp8":
            self.k_cache = torch.zeros(shape_k, device=self.device, dtype=torch.uint8).view(torch.float8_e4m3fn)
            self.v_cache = torch.zeros(shape_v, device=self.device, dtype=torch.uint8).view(torch.float8_e4m3fn)
        else:
            self.k_cache = torch.zeros(shape_k, device=self.device, dtype=self.dtype)
            self.v_cache = torch.zeros(shape_v, device=self.device, dtype=self.dtype)
        return self.k_cache, self.v_cache

    def copy_kv_blocks(self, src: torch.Tensor, dst: torch.Tensor) -> None:
        """Copy-on-fork (beam search): page ``dst[i]`` of every layer takes the K and Vᵀ of
        page ``src[i]`` — one gather/scatter per cache over the [layers, blocks] dims."""
        src, dst = src.to(self.device).long(), dst.to(self.device).long()
        for c in (self.k_cache, self.v_cache):
            raw = c.view(torch.uint8) if c.dtype == torch.float8_e4m3fn else c
            raw.index_copy_(1, dst, raw.index_select(1, src))

    def kv_block_bytes(self, block_size: int = 64, kv_dtype: str = "auto") -> int:
        elem = 1 if kv_dtype == "fp8" else torch.finfo(self.dtype).bits // 8
        return 2 * len(self.layers) * self.hkv * self.D * block_size * elem

    # ------------------------------------------------------------------ forward
    def embed_tokens(self, ids: torch.Tensor) -> torch.Tensor:
        """Vocab-parallel embedding (K8, CC3): each rank gathers the rows of its vocabulary
        shard (zeros elsewhere) and the TP all-reduce sums them. Gemma's embedding scale is
        a bf16 constant (HF multiplies by it in the model dtype); the gather applies it."""
        lo = self.p.tp_rank * self.vocab_local if self.p.tp_size > 1 else 0
        if self.embed.dtype == torch.bfloat16 or not ids.is_cuda:
            h = ops.embedding(ids, self.embed, lo, self.cfg.embed_scale)
        else:   # fp32 tables (CPU-reference models moved to the GPU)
            h = ref.embedding(ids, self.embed, lo, self.cfg.embed_scale)
        if self.p.tp_size > 1:
            h = tp_all_reduce(h, self.p)
        return h

    # norms: RMSNorm (Llama/Mistral/Mixtral/Gemma) or LayerNorm with bias (StarCoder2)
    def _norm(self, x, w, b=None):
        if b is None:
            return ops.rmsnorm(x, w, self.cfg.eps)
        return ops.layernorm(x, w, b, self.cfg.eps)

    def _add_norm(self, resid, delta, w, b=None):
        """resid += delta (in place); returns norm(resid)."""
        if b is None:
            return ops.add_rmsnorm(resid, delta, w, self.cfg.eps)
        return ops.add_layernorm(resid, delta, w, b, self.cfg.eps)

    def _bias_rank0(self, y: torch.Tensor, b: Optional[torch.Tensor]) -> torch.Tensor:
        """A row-parallel projection's bias joins the TP partial sum on one rank only."""
        if b is not None and self.p.tp_rank == 0:
            y.add_(b)
        return y

    def _qkv(self, x, L, partial_ok: bool = False):
        if "bqkv" in L:
            return torch.addmm(L["bqkv"], x, L["wqkv"].t())
        return self._lin(x, L, "wqkv", partial_ok=partial_ok)

    @staticmethod
    def _gemv_ok(x, w) -> bool:
        return (x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.is_contiguous()
                and x.stride(1) == 1 and x.stride(0) % 8 == 0 and x.shape[1] % 8 == 0
                and x.shape[0] * x.shape[1] * 2 <= 160 * 1024)

    def _mlp(self, x, L, partial_ok: bool = False):
        """MLP of one layer on normed rows; returns the (TP partial) output (an
        ``ops.PartialSum`` of K-split slabs when ``partial_ok`` and the down GEMM split K)."""
        cfg = self.cfg
        if cfg.is_moe:
            return ops.moe_ffn(x, L["router"], L["w13"], L["w2"], cfg.experts_per_tok,
                               expert0=self.expert0, act=cfg.act, ws=self.moe_ws)
        if cfg.gated_mlp:
            if cfg.act == "silu":
                if self.skinny and "wgu" in L and x.shape[0] <= ops.GEMV_MAX_M and self._gemv_ok(x, L["wgu"]):
                    # 1-4 rows: weight-streaming GEMV with the SwiGLU epilogue (5.0-5.8 TB/s)
                    return self._lin(ops.gemv(x, L["wgu"], 2), L, "wd", partial_ok=partial_ok)
                pk = self._pick(L["wgu"], x.shape[0]) if "wgu" in L else None
                if pk is not None:   # SwiGLU in the gate|up GEMM's epilogue: [M, F] straight out
                    if pk[1] == 1:
                        h = ops.skinny_gemm(x, L["wgu"], pk[0], 1, 2)
                    else:            # K split: the SwiGLU kernel sums the fp32 slabs
                        h = ops.splitk_swiglu(ops.skinny_gemm(x, L["wgu"], pk[0], pk[1], 1))
                    return self._lin(h, L, "wd", partial_ok=partial_ok)
            gu = self._lin(x, L, "wgu")
            if cfg.act == "silu":
                return self._lin(gu, L, "wd", swiglu=True, partial_ok=partial_ok)
            return self._lin(ops.gelu_tanh_mul(gu), L, "wd", partial_ok=partial_ok)
        h = x @ L["wgu"].t()
        ops.bias_gelu_(h, L.get("bgu"), approximate=cfg.act == "gelu_tanh")
        return self._bias_rank0(h @ L["wd"].t(), L.get("bd"))

    def _attention(self, q, qkv, li, meta: AttnMeta, T: int):
        hq, hkv, D = self.hq, self.hkv, self.D
        qdim = hq * D
        W = self.window
        if meta.kind == "decode":
            return ops.decode_attention(q, self.k_cache[li], self.v_cache[li],
                                        meta.block_tables, meta.ctx_lens, hq, hkv,
                                        meta.max_ctx, self.scale, ws=meta.decode_ws, window=W,
                                        kv_scales=self.kv_scales)
        if meta.kind == "graph":
            return self._attention_graph(q, qkv, li, meta, T)
        if meta.kind == "mixed":
            nd = meta.n_decode
            attn = torch.empty(T, qdim, dtype=qkv.dtype, device=qkv.device)

            def prefill():
                ops.prefill_attention_paged(q[nd:], self.k_cache[li], self.v_cache[li],
                                            meta.block_tables[nd:], meta.cu_q_prefill,
                                            meta.ctx_lens[nd:], hq, hkv, D, meta.max_q_len,
                                            self.scale, out=attn[nd:], window=W,
                                            kv_scales=self.kv_scales)

            side = None
            if self.concurrent_attention and qkv.is_cuda and not torch.cuda.is_current_stream_capturing():
                if self._attn_stream is None:
                    self._attn_stream = torch.cuda.Stream(qkv.device)
                side = self._attn_stream
                main = torch.cuda.current_stream(qkv.device)
                side.wait_stream(main)           # q / K / V pages written on main
                with torch.cuda.stream(side):
                    prefill()
            ops.decode_attention(q[:nd], self.k_cache[li], self.v_cache[li],
                                 meta.block_tables[:nd], meta.ctx_lens[:nd], hq, hkv,
                                 meta.max_ctx, self.scale, out=attn[:nd], ws=meta.decode_ws,
                                 window=W, kv_scales=self.kv_scales)
            if side is not None:
                main.wait_stream(side)           # attn (allocated on main) complete
            else:
                prefill()
            return attn
        # a prefill-only step: no decode attention shares the chip (impl 4)
        return ops.prefill_attention_paged(q, self.k_cache[li], self.v_cache[li],
                                           meta.block_tables, meta.cu_q, meta.ctx_lens,
                                           hq, hkv, D, meta.max_q_len, self.scale, window=W,
                                           kv_scales=self.kv_scales, impl=4)

    def _attention_graph(self, q, qkv, li, meta: AttnMeta, T: int):
        """Attention of a graph-captured step: the decode launch over the bucket's first
        n_decode rows (rows whose decode_ctx is 0 are not this step's and stay untouched) on
        the current stream and the work-list prefill kernel on the side stream, writing
        disjoint rows of one output (rows no one covers are bucket padding)."""
        hq, hkv, D = self.hq, self.hkv, self.D
        W = self.window
        attn = torch.empty(T, hq * D, dtype=qkv.dtype, device=qkv.device)
        nd = meta.n_decode
        if meta.pf_seq:   # back to back on the current stream: decode rows, then the work list
            if nd:
                ops.decode_attention(q[:nd], self.k_cache[li], self.v_cache[li], meta.block_tables[:nd],
                                     meta.decode_ctx[:nd], hq, hkv, meta.max_ctx, self.scale, out=attn[:nd],
                                     ws=meta.decode_ws, window=W, kv_scales=self.kv_scales, skip_empty=True)
            ops.prefill_attention_worklist(q, self.k_cache[li], self.v_cache[li], meta.block_tables, meta.cu_q,
                                           meta.ctx_lens, hq, hkv, self.scale, meta.items, meta.n_items,
                                           grid=meta.pf_grid, ks=meta.pf_ks, out=attn, window=W,
                                           impl=meta.pf_impl, kv_scales=self.kv_scales)
            return attn
        gpu = qkv.is_cuda
        if gpu:
            if self._attn_stream is None:
                self._attn_stream = torch.cuda.Stream(qkv.device)
            side = self._attn_stream
            main = torch.cuda.current_stream(qkv.device)
            side.wait_stream(main)
        with (torch.cuda.stream(side) if gpu else contextlib.nullcontext()):
            ops.prefill_attention_worklist(q, self.k_cache[li], self.v_cache[li], meta.block_tables, meta.cu_q,
                                           meta.ctx_lens, hq, hkv, self.scale, meta.items, meta.n_items,
                                           grid=meta.pf_grid, ks=meta.pf_ks, out=attn, window=W,
                                           impl=meta.pf_impl, kv_scales=self.kv_scales)
        if nd:
            ops.decode_attention(q[:nd], self.k_cache[li], self.v_cache[li], meta.block_tables[:nd],
                                 meta.decode_ctx[:nd], hq, hkv, meta.max_ctx, self.scale, out=attn[:nd],
                                 ws=meta.decode_ws, window=W, kv_scales=self.kv_scales, skip_empty=True)
        if gpu:
            main.wait_stream(side)
        return attn

    def _reduce_add_norm(self, partial, resid, w, b=None):
        """resid += all_reduce_TP(partial); returns norm(resid). A small TP message goes
        through the custom all-reduce's fused add+RMSNorm epilogue kernel (one launch, the
        sum never round-trips through HBM); otherwise all-reduce, then the add+norm kernel.
        K-split skinny partials (one rank) are summed inside the add+RMSNorm kernel."""
        if isinstance(partial, ops.PartialSum):
            if b is None and self.p.tp_size == 1:
                return ops.splitk_add_rmsnorm(resid, partial.slabs, w, self.cfg.eps)
            partial = partial.materialize()
        if self.p.tp_size > 1:
            car = custom_all_reduce_for(self.p.tp_group)
            if b is None and car is not None and car.fused_norm_eligible(partial):
                return car.all_reduce_add_rmsnorm(partial, resid, w, self.cfg.eps)
            tp_all_reduce(partial, self.p)
        return self._add_norm(resid, partial, w, b)

    def _attn_block(self, li: int, x, pos, meta: AttnMeta, T: int, partial_ok: bool = False):
        """qkv projection + RoPE/KV write + attention + o projection (TP partial; an
        ``ops.PartialSum`` when ``partial_ok`` and the o GEMM split K)."""
        L = self.layers[li]
        qkv = self._qkv(x, L, partial_ok=True)
        part = None
        if isinstance(qkv, ops.PartialSum):   # K-split projection: the RoPE kernel sums the slabs
            part = qkv
            qkv = torch.empty(part.shape, dtype=x.dtype, device=x.device)
        ops.rope_cache_(qkv, pos, self.cos_sin, meta.slots, self.k_cache[li],
                        self.v_cache[li], self.hq, self.hkv, self.D, kv_scales=self.kv_scales, partial=part)
        attn = self._attention(qkv[:, :self.hq * self.D], qkv, li, meta, T)
        if "bo" in L:
            return self._bias_rank0(self._lin(attn, L, "wo"), L.get("bo"))
        return self._lin(attn, L, "wo", partial_ok=partial_ok)

    def _layer(self, li: int, x, resid, pos, meta: AttnMeta):
        """One decoder layer on rows (x = norm(resid)); returns the MLP output d — still
        a TP partial sum — which the caller reduces into resid with the next layer's (or
        the final) norm."""
        L = self.layers[li]
        o = self._attn_block(li, x, pos, meta, x.shape[0], partial_ok=True)
        x = self._reduce_add_norm(o, resid, L["mlp_norm"], L.get("mlp_norm_b"))
        return self._mlp(x, L, partial_ok="bd" not in L)

    def _final(self, resid, d, sample_idx):
        """Final norm of resid + d (all rows, or only the sampling rows)."""
        if sample_idx is not None:
            rows = resid.index_select(0, sample_idx) + d.index_select(0, sample_idx)
            return self._norm(rows.contiguous(), self.final_norm, self.final_norm_b)
        return self._add_norm(resid, d, self.final_norm, self.final_norm_b)

    def _stack(self, resid, pos, meta: AttnMeta, sample_idx: Optional[torch.Tensor]):
        L0 = self.layers[0]
        x = self._norm(resid, L0["attn_norm"], L0.get("attn_norm_b"))
        n = len(self.layers)
        for li in range(n):
            d = self._layer(li, x, resid, pos, meta)
            if li + 1 < n:
                Ln = self.layers[li + 1]
                x = self._reduce_add_norm(d, resid, Ln["attn_norm"], Ln.get("attn_norm_b"))
                continue
            if isinstance(d, ops.PartialSum):
                d = d.materialize()
            tp_all_reduce(d, self.p)
            return self._final(resid, d, sample_idx)
        raise RuntimeError("model has no layers")

    def forward(self, ids: torch.Tensor, pos: torch.Tensor, meta: AttnMeta,
                sample_idx: Optional[torch.Tensor] = None, embed_override=None) -> torch.Tensor:
        """Returns the final-normed hidden rows selected by ``sample_idx`` (all rows if None).
        With pipeline stages only stage 0 gets them (other stages return None).
        ``embed_override = (rows, features)`` replaces those rows' input embeddings (the
        projected image patches of a vision-language prompt)."""
        if self.p.pp_size > 1:
            return self._forward_pp(ids, pos, meta, sample_idx, embed_override)
        if (self.sequence_parallel and self.p.tp_size > 1 and meta.kind == "prefill"
                and ids.shape[0] >= self.sp_min_tokens and embed_override is None):
            return self._forward_sp(ids, pos, meta, sample_idx)
        if (meta.kind == "mixed" and self.split_mixed and ids.is_cuda and self.p.tp_size == 1
                and embed_override is None):
            return self.forward_split(ids, pos, meta, sample_idx)
        return self._stack(self._embed(ids, embed_override), pos, meta, sample_idx)

    def _embed(self, ids, embed_override=None):
        h = self.embed_tokens(ids)
        if embed_override is not None:
            rows, feats = embed_override
            h.index_copy_(0, rows, feats.to(h.dtype))
        return h

    def _forward_sp(self, ids, pos, meta: AttnMeta, sample_idx):
        """Megatron-style sequence parallelism inside the TP group for long prefills: the
        residual stream and both RMSNorms live on this rank's T / tp rows; each column-
        parallel GEMM is preceded by an all-gather of the normed rows and each row-parallel
        GEMM followed by a reduce-scatter, which together move the bytes of the all-reduce
        they replace while the norm/residual work and activation memory drop by tp x.
        Rows are padded to a multiple of tp (padding rows write no KV: slot -1)."""
        cfg, p = self.cfg, self.p
        tp, r = p.tp_size, p.tp_rank
        self.sp_steps += 1
        T = ids.shape[0]
        Tp = -(-T // tp) * tp
        if Tp != T:
            pad = Tp - T
            ids = torch.cat([ids, ids.new_zeros(pad)])
            pos = torch.cat([pos, pos.new_zeros(pad)])
            slots = torch.cat([meta.slots, meta.slots.new_full((pad,), -1)])
            meta = AttnMeta(kind=meta.kind, slots=slots, cu_q=meta.cu_q, ctx_lens=meta.ctx_lens,
                            block_tables=meta.block_tables, max_q_len=meta.max_q_len,
                            max_ctx=meta.max_ctx, decode_ws=meta.decode_ws)
        # vocab-parallel embedding: partial rows, reduce-scattered straight into the shard
        lo = r * self.vocab_local
        local = ids.long() - lo
        ok = (local >= 0) & (local < self.vocab_local)
        h = torch.nn.functional.embedding(local.clamp(0, self.vocab_local - 1), self.embed)
        resid = tp_reduce_scatter_rows(h * ok.unsqueeze(-1).to(h.dtype), p).contiguous()
        if cfg.embed_scale != 1.0:
            resid = resid * torch.tensor(cfg.embed_scale, dtype=resid.dtype)
        L0 = self.layers[0]
        x = self._norm(resid, L0["attn_norm"], L0.get("attn_norm_b"))
        n = len(self.layers)
        d = None
        for li in range(n):
            L = self.layers[li]
            xf = tp_all_gather_rows(x, p)
            o = tp_reduce_scatter_rows(self._attn_block(li, xf, pos, meta, Tp), p).contiguous()
            x = self._add_norm(resid, o, L["mlp_norm"], L.get("mlp_norm_b"))
            d = tp_reduce_scatter_rows(self._mlp(tp_all_gather_rows(x, p), L), p).contiguous()
            if li + 1 < n:
                Ln = self.layers[li + 1]
                x = self._add_norm(resid, d, Ln["attn_norm"], Ln.get("attn_norm_b"))
        out = tp_all_gather_rows(self._add_norm(resid, d, self.final_norm, self.final_norm_b), p)[:T]
        return out if sample_idx is None else out.index_select(0, sample_idx)

    def _forward_pp(self, ids, pos, meta: AttnMeta, sample_idx, embed_override=None):
        """Layer-split pipeline (SURVEY.md §2.E "PP", CC6): stage s receives the residual
        stream from stage s-1, runs its layers and sends it on (RCCL p2p over xGMI); the
        last stage applies the final norm to the sampling rows and returns them to stage 0,
        which owns the LM head and samples. One step flows through the stages in turn — the
        reference's HF ``device_map="auto"`` layer placement (examples/multimodal_rag/llm/
        llm.py:42-47), for models that outgrow one GPU's HBM without a TP group."""
        import torch.distributed as dist

        cfg, p = self.cfg, self.p
        T = ids.shape[0]
        if self.first_stage:
            resid = self._embed(ids, embed_override)
        else:
            resid = torch.empty(T, cfg.hidden, dtype=self.dtype, device=self.device)
            dist.recv(resid, src=p.pp_prev)
        L0 = self.layers[0]
        x = self._norm(resid, L0["attn_norm"], L0.get("attn_norm_b"))
        n = len(self.layers)
        for li in range(n):
            d = self._layer(li, x, resid, pos, meta)
            if li + 1 < n:
                Ln = self.layers[li + 1]
                x = self._reduce_add_norm(d, resid, Ln["attn_norm"], Ln.get("attn_norm_b"))
        if isinstance(d, ops.PartialSum):
            d = d.materialize()
        tp_all_reduce(d, self.p)
        rows = T if sample_idx is None else int(sample_idx.shape[0])
        if not self.last_stage:
            resid.add_(d)
            dist.send(resid, dst=p.pp_next)
            h = None
        else:
            h = self._final(resid, d, sample_idx)
            dist.send(h.contiguous(), dst=p.pp_first_rank)
            h = None
        if self.first_stage:
            h = torch.empty(rows, cfg.hidden, dtype=self.dtype, device=self.device)
            dist.recv(h, src=p.pp_last_rank)
        return h

    def forward_split(self, ids: torch.Tensor, pos: torch.Tensor, meta: AttnMeta,
                      sample_idx: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Mixed step as two independent row groups on two HIP streams: the decode rows
        (memory-bound: paged-KV attention streams ~1.4 GB per layer at 256 x 1400) on an
        auxiliary stream, the prefill chunk (compute-bound GEMMs) on the current stream.
        The groups share no data inside the stack — each writes the KV pages of its own
        sequences — so the GPU co-schedules them for all layers and the KV stream of the
        decode rows fills the CUs that the prefill GEMMs' tile grid leaves idle.
        ``sample_idx`` must list the decode rows first (the engine's layout).

        Measured on MI355X (benchmarks/mixed_step.py, profiles/r1_mixed_split): 256 decode
        rows x 1330 ctx + a 1170-token chunk takes 31.1 ms split vs 28.5 ms fused (2048-token
        chunk: 38.9 vs 37.8 ms). hipBLASLt's stream-K GEMMs occupy every CU, so the decode
        attention gets no idle CUs to run on while the split costs GEMM efficiency (M=256 and
        M=1170 instead of one M=1426 GEMM). Off by default (``split_mixed``)."""
        nd = meta.n_decode
        main = torch.cuda.current_stream(ids.device)
        if self._aux is None:
            self._aux = torch.cuda.Stream(ids.device)
        aux = self._aux
        resid = self.embed_tokens(ids)
        md = AttnMeta(kind="decode", slots=meta.slots[:nd], cu_q=meta.cu_q[:nd + 1],
                      ctx_lens=meta.ctx_lens[:nd], block_tables=meta.block_tables[:nd],
                      max_q_len=1, max_ctx=meta.max_ctx, decode_ws=meta.decode_ws)
        mp = AttnMeta(kind="prefill", slots=meta.slots[nd:], cu_q=meta.cu_q_prefill,
                      ctx_lens=meta.ctx_lens[nd:], block_tables=meta.block_tables[nd:],
                      max_q_len=meta.max_q_len, max_ctx=meta.max_ctx)
        aux.wait_stream(main)
        with torch.cuda.stream(aux):
            hd = self._stack(resid[:nd], pos[:nd], md, None)
        sp = None if sample_idx is None else sample_idx[nd:] - nd
        hp = self._stack(resid[nd:], pos[nd:], mp, sp)
        main.wait_stream(aux)
        hd.record_stream(main)
        resid.record_stream(aux)
        return torch.cat([hd, hp])

    def ipc_collectives_cover(self, rows: int, tokens: int) -> bool:
        """True when every collective of a forward over ``tokens`` token rows that samples
        ``rows`` rows goes through the TP group's IPC custom kernels (all-reduces of [tokens,
        hidden] bf16, the [rows, vocab / tp] fp32 logits all-gather), which a hipGraph can
        hold whatever the process-group backend (gloo's host-copy collectives it cannot)."""
        if self.p.tp_size == 1:
            return True
        car = custom_all_reduce_for(self.p.tp_group)
        if car is None or not car.enabled or self.expert_parallel:
            return False
        ar = tokens * self.cfg.hidden * 2
        ag = rows * self.vocab_local * 4
        return (ar <= car.capacity and ag <= car.capacity and (self.cfg.hidden * 2) % 16 == 0
                and (self.vocab_local * 4) % 16 == 0)

    def logits(self, h: torch.Tensor) -> torch.Tensor:
        """fp32 logits over the full vocabulary (vocab-parallel head + all-gather). Where the
        skinny table picks it, the LM head GEMM writes fp32 straight from its accumulators
        (no bf16 logits tensor and no conversion pass)."""
        ok = (self.skinny and h.is_cuda and h.dtype == torch.bfloat16 and self.lm_head.dtype == torch.bfloat16
              and h.stride(1) == 1 and h.stride(0) % 8 == 0)
        pk = self._pick(self.lm_head, h.shape[0]) if ok else None
        if ok and h.shape[0] <= ops.GEMV_MAX_M and self.lm_head.is_contiguous():
            # 1-4 rows (batch-1..4 decode): the weight-streaming GEMV (6.4 TB/s vs 5.9 library)
            lg = ops.gemv(h, self.lm_head, 1)
        elif pk is not None and pk[1] == 1:
            lg = ops.skinny_gemm(h, self.lm_head, pk[0], 1, 1)[0]
        else:
            lg = (h @ self.lm_head.t()).float()
        return tp_all_gather(lg, dim=-1, ctx=self.p)


# family-neutral name
DecoderModel = LlamaModel
