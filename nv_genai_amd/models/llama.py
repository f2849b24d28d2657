"""Llama-3 decoder (8B / 70B) on the gfx950 kernel set, tensor-parallel over RCCL.

This is the MI355X-native replacement for the TensorRT-LLM engine inside NIM
(SURVEY.md §2.B N1). Per layer:

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
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

from .. import ops
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


class LlamaModel:
    def __init__(self, cfg: LlamaConfig, device="cuda", dtype=torch.bfloat16,
                 pctx: Optional[ParallelContext] = None, seed: int = 0,
                 weights: Optional[Dict[str, torch.Tensor]] = None, fp8: bool = False):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.p = pctx or get_context()
        tp = self.p.tp_size
        if cfg.heads % tp or cfg.kv_heads % tp or cfg.ffn % tp or cfg.vocab_size % tp:
            raise ValueError(f"{cfg.name}: dims not divisible by tp={tp}")
        self.hq = cfg.heads // tp
        self.hkv = cfg.kv_heads // tp
        self.D = cfg.head_dim
        self.ffn = cfg.ffn // tp
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
        for L in self.layers:
            for n in self._LINEARS:
                L[n + "8"], L[n + "_s"] = ops.quantize_weight_fp8(L.pop(n))
        self.fp8 = True
        if self.device.type == "cuda":
            torch.cuda.empty_cache()

    def _lin(self, x: torch.Tensor, L: dict, name: str, swiglu: bool = False) -> torch.Tensor:
        """x @ W^T for projection ``name`` (bf16, or FP8 W8A8 when quantised); ``swiglu``:
        x is the [M, 2F] gate|up output and the projection consumes silu(gate) * up."""
        if not self.fp8:
            return (ops.silu_mul(x) if swiglu else x) @ L[name].t()
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

        g.manual_seed(seed * 1000 + self.p.tp_rank)
        out_std = 0.02 / math.sqrt(2 * cfg.layers)
        reseed(0)
        self.embed = rnd(self.vocab_local, H) if self.first_stage else None
        self.layers: List[Dict[str, torch.Tensor]] = []
        for i in range(self.layer_lo, self.layer_hi):
            reseed(i + 2)
            self.layers.append({
                "attn_norm": torch.ones(H, device=dev, dtype=dt),
                "wqkv": rnd((self.hq + 2 * self.hkv) * self.D, H),
                "wo": rnd(H, self.hq * self.D, std=out_std),
                "mlp_norm": torch.ones(H, device=dev, dtype=dt),
                "wgu": rnd(2 * self.ffn, H),
                "wd": rnd(H, self.ffn, std=out_std),
            })
        self.final_norm = torch.ones(H, device=dev, dtype=dt)
        reseed(1)
        self.lm_head = rnd(self.vocab_local, H) if self.first_stage else None

    def _load(self, w: Dict[str, torch.Tensor]):
        """Load HF-named Llama weights (model.layers.N.self_attn.q_proj.weight, ...),
        fusing q/k/v and gate/up, and slicing this rank's TP shard."""
        cfg, dev, dt = self.cfg, self.device, self.dtype
        tp, r = self.p.tp_size, self.p.tp_rank

        def rows(t, n):  # column-parallel shard (output rows)
            c = t.shape[0] // tp
            return t[r * c:(r + 1) * c]

        def cols(t):  # row-parallel shard (input columns)
            c = t.shape[1] // tp
            return t[:, r * c:(r + 1) * c]

        def get(name):
            return w[name].to(dev, dt)

        self.embed = rows(get("model.embed_tokens.weight"), 0).contiguous() if self.first_stage else None
        self.layers = []
        for i in range(self.layer_lo, self.layer_hi):
            p = f"model.layers.{i}."
            q, k, v = get(p + "self_attn.q_proj.weight"), get(p + "self_attn.k_proj.weight"), get(p + "self_attn.v_proj.weight")
            gt, up = get(p + "mlp.gate_proj.weight"), get(p + "mlp.up_proj.weight")
            self.layers.append({
                "attn_norm": get(p + "input_layernorm.weight"),
                "wqkv": torch.cat([rows(q, 0), rows(k, 0), rows(v, 0)]).contiguous(),
                "wo": cols(get(p + "self_attn.o_proj.weight")).contiguous(),
                "mlp_norm": get(p + "post_attention_layernorm.weight"),
                "wgu": torch.cat([rows(gt, 0), rows(up, 0)]).contiguous(),
                "wd": cols(get(p + "mlp.down_proj.weight")).contiguous(),
            })
        self.final_norm = get("model.norm.weight")
        self.lm_head = None
        if self.first_stage:
            head = w.get("lm_head.weight", w["model.embed_tokens.weight"]).to(dev, dt)
            self.lm_head = rows(head, 0).contiguous()

    def state_dict(self) -> Dict[str, torch.Tensor]:
        """HF-named weights of this rank (unfused; TP shards are local slices; a pipeline
        stage holds only its layers, plus embedding and LM head on stage 0)."""
        if self.fp8:
            raise RuntimeError("state_dict of an FP8-quantised model: export the bf16 model before quantize_fp8()")
        out = {"model.norm.weight": self.final_norm}
        if self.first_stage:
            out["model.embed_tokens.weight"] = self.embed
            out["lm_head.weight"] = self.lm_head
        qd, kd = self.hq * self.D, self.hkv * self.D
        for i, L in enumerate(self.layers, start=self.layer_lo):
            p = f"model.layers.{i}."
            out[p + "input_layernorm.weight"] = L["attn_norm"]
            out[p + "self_attn.q_proj.weight"] = L["wqkv"][:qd]
            out[p + "self_attn.k_proj.weight"] = L["wqkv"][qd:qd + kd]
            out[p + "self_attn.v_proj.weight"] = L["wqkv"][qd + kd:]
            out[p + "self_attn.o_proj.weight"] = L["wo"]
            out[p + "post_attention_layernorm.weight"] = L["mlp_norm"]
            out[p + "mlp.gate_proj.weight"] = L["wgu"][: self.ffn]
            out[p + "mlp.up_proj.weight"] = L["wgu"][self.ffn:]
            out[p + "mlp.down_proj.weight"] = L["wd"]
        return out

    # ------------------------------------------------------------------ cache
    def allocate_kv_cache(self, num_blocks: int, block_size: int = 64):
        if block_size != 64:
            raise ValueError("the gfx950 attention kernels use 64-token KV pages")
        shape_k = (len(self.layers), num_blocks, self.hkv, block_size, self.D)
        shape_v = (len(self.layers), num_blocks, self.hkv, self.D, block_size)
        # zero-filled: masked keys of a partially filled page must stay finite
        self.k_cache = torch.zeros(shape_k, device=self.device, dtype=self.dtype)
        self.v_cache = torch.zeros(shape_v, device=self.device, dtype=self.dtype)
        return self.k_cache, self.v_cache

    def copy_kv_blocks(self, src: torch.Tensor, dst: torch.Tensor) -> None:
        """Copy-on-fork (beam search): page ``dst[i]`` of every layer takes the K and Vᵀ of
        page ``src[i]`` — one gather/scatter per cache over the [layers, blocks] dims."""
        src, dst = src.to(self.device).long(), dst.to(self.device).long()
        self.k_cache.index_copy_(1, dst, self.k_cache.index_select(1, src))
        self.v_cache.index_copy_(1, dst, self.v_cache.index_select(1, src))

    def kv_block_bytes(self, block_size: int = 64) -> int:
        return 2 * len(self.layers) * self.hkv * self.D * block_size * torch.finfo(self.dtype).bits // 8

    # ------------------------------------------------------------------ forward
    def embed_tokens(self, ids: torch.Tensor) -> torch.Tensor:
        if self.p.tp_size == 1:
            return torch.nn.functional.embedding(ids.long(), self.embed)
        lo = self.p.tp_rank * self.vocab_local
        local = ids.long() - lo
        ok = (local >= 0) & (local < self.vocab_local)
        h = torch.nn.functional.embedding(local.clamp(0, self.vocab_local - 1), self.embed)
        h = h * ok.unsqueeze(-1).to(h.dtype)
        return tp_all_reduce(h, self.p)

    def _attention(self, q, qkv, li, meta: AttnMeta, T: int):
        hq, hkv, D = self.hq, self.hkv, self.D
        qdim = hq * D
        if meta.kind == "decode":
            return ops.decode_attention(q, self.k_cache[li], self.v_cache[li],
                                        meta.block_tables, meta.ctx_lens, hq, hkv,
                                        meta.max_ctx, self.scale, ws=meta.decode_ws)
        if meta.kind == "mixed":
            nd = meta.n_decode
            attn = torch.empty(T, qdim, dtype=qkv.dtype, device=qkv.device)

            def prefill():
                ops.prefill_attention_paged(q[nd:], self.k_cache[li], self.v_cache[li],
                                            meta.block_tables[nd:], meta.cu_q_prefill,
                                            meta.ctx_lens[nd:], hq, hkv, D, meta.max_q_len,
                                            self.scale, out=attn[nd:])

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
                                 meta.max_ctx, self.scale, out=attn[:nd], ws=meta.decode_ws)
            if side is not None:
                main.wait_stream(side)           # attn (allocated on main) complete
            else:
                prefill()
            return attn
        return ops.prefill_attention_paged(q, self.k_cache[li], self.v_cache[li],
                                           meta.block_tables, meta.cu_q, meta.ctx_lens,
                                           hq, hkv, D, meta.max_q_len, self.scale)

    def _reduce_add_norm(self, partial, resid, w):
        """resid += all_reduce_TP(partial); returns rmsnorm(resid) * w. A small TP message
        goes through the custom all-reduce's fused epilogue kernel (one launch, the sum never
        round-trips through HBM); otherwise all-reduce, then the add+RMSNorm kernel."""
        if self.p.tp_size > 1:
            car = custom_all_reduce_for(self.p.tp_group)
            if car is not None and car.fused_norm_eligible(partial):
                return car.all_reduce_add_rmsnorm(partial, resid, w, self.cfg.eps)
            tp_all_reduce(partial, self.p)
        return ops.add_rmsnorm(resid, partial, w, self.cfg.eps)

    def _layer(self, li: int, x, resid, pos, meta: AttnMeta):
        """One decoder layer on rows (x = rmsnorm(resid)); returns the MLP output d — still
        a TP partial sum — which the caller reduces into resid with the next layer's (or
        the final) norm."""
        L = self.layers[li]
        qkv = self._lin(x, L, "wqkv")
        ops.rope_cache_(qkv, pos, self.cos_sin, meta.slots, self.k_cache[li],
                        self.v_cache[li], self.hq, self.hkv, self.D)
        attn = self._attention(qkv[:, :self.hq * self.D], qkv, li, meta, x.shape[0])
        o = self._lin(attn, L, "wo")
        x = self._reduce_add_norm(o, resid, L["mlp_norm"])
        return self._lin(self._lin(x, L, "wgu"), L, "wd", swiglu=True)

    def _stack(self, resid, pos, meta: AttnMeta, sample_idx: Optional[torch.Tensor]):
        cfg = self.cfg
        x = ops.rmsnorm(resid, self.layers[0]["attn_norm"], cfg.eps)
        n = len(self.layers)
        for li in range(n):
            d = self._layer(li, x, resid, pos, meta)
            if li + 1 < n:
                x = self._reduce_add_norm(d, resid, self.layers[li + 1]["attn_norm"])
                continue
            tp_all_reduce(d, self.p)
            if sample_idx is not None:
                # only rows that sample need the final norm
                rows = resid.index_select(0, sample_idx) + d.index_select(0, sample_idx)
                return ops.rmsnorm(rows.contiguous(), self.final_norm, cfg.eps)
            else:
                return ops.add_rmsnorm(resid, d, self.final_norm, cfg.eps)
        raise RuntimeError("model has no layers")

    def forward(self, ids: torch.Tensor, pos: torch.Tensor, meta: AttnMeta,
                sample_idx: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Returns the final-normed hidden rows selected by ``sample_idx`` (all rows if None).
        With pipeline stages only stage 0 gets them (other stages return None)."""
        if self.p.pp_size > 1:
            return self._forward_pp(ids, pos, meta, sample_idx)
        if (self.sequence_parallel and self.p.tp_size > 1 and meta.kind == "prefill"
                and ids.shape[0] >= self.sp_min_tokens):
            return self._forward_sp(ids, pos, meta, sample_idx)
        if meta.kind == "mixed" and self.split_mixed and ids.is_cuda and self.p.tp_size == 1:
            return self.forward_split(ids, pos, meta, sample_idx)
        return self._stack(self.embed_tokens(ids), pos, meta, sample_idx)

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
        rows = Tp // tp
        # vocab-parallel embedding: partial rows, reduce-scattered straight into the shard
        lo = r * self.vocab_local
        local = ids.long() - lo
        ok = (local >= 0) & (local < self.vocab_local)
        h = torch.nn.functional.embedding(local.clamp(0, self.vocab_local - 1), self.embed)
        resid = tp_reduce_scatter_rows(h * ok.unsqueeze(-1).to(h.dtype), p).contiguous()
        x = ops.rmsnorm(resid, self.layers[0]["attn_norm"], cfg.eps)
        n = len(self.layers)
        d = None
        for li in range(n):
            L = self.layers[li]
            xf = tp_all_gather_rows(x, p)
            qkv = self._lin(xf, L, "wqkv")
            ops.rope_cache_(qkv, pos, self.cos_sin, meta.slots, self.k_cache[li],
                            self.v_cache[li], self.hq, self.hkv, self.D)
            attn = self._attention(qkv[:, :self.hq * self.D], qkv, li, meta, Tp)
            o = tp_reduce_scatter_rows(self._lin(attn, L, "wo"), p).contiguous()
            x = ops.add_rmsnorm(resid, o, L["mlp_norm"], cfg.eps)
            gu = self._lin(tp_all_gather_rows(x, p), L, "wgu")
            d = tp_reduce_scatter_rows(self._lin(gu, L, "wd", swiglu=True), p).contiguous()
            if li + 1 < n:
                x = ops.add_rmsnorm(resid, d, self.layers[li + 1]["attn_norm"], cfg.eps)
        out = tp_all_gather_rows(ops.add_rmsnorm(resid, d, self.final_norm, cfg.eps), p)[:T]
        return out if sample_idx is None else out.index_select(0, sample_idx)

    def _forward_pp(self, ids, pos, meta: AttnMeta, sample_idx):
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
            resid = self.embed_tokens(ids)
        else:
            resid = torch.empty(T, cfg.hidden, dtype=self.dtype, device=self.device)
            dist.recv(resid, src=p.pp_prev)
        x = ops.rmsnorm(resid, self.layers[0]["attn_norm"], cfg.eps)
        n = len(self.layers)
        for li in range(n):
            d = self._layer(li, x, resid, pos, meta)
            if li + 1 < n:
                x = self._reduce_add_norm(d, resid, self.layers[li + 1]["attn_norm"])
        tp_all_reduce(d, self.p)
        rows = T if sample_idx is None else int(sample_idx.shape[0])
        if not self.last_stage:
            resid.add_(d)
            dist.send(resid, dst=p.pp_next)
            h = None
        else:
            if sample_idx is not None:
                r = resid.index_select(0, sample_idx) + d.index_select(0, sample_idx)
                h = ops.rmsnorm(r.contiguous(), self.final_norm, cfg.eps)
            else:
                h = ops.add_rmsnorm(resid, d, self.final_norm, cfg.eps)
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

    def logits(self, h: torch.Tensor) -> torch.Tensor:
        """fp32 logits over the full vocabulary (vocab-parallel head + all-gather)."""
        lg = (h @ self.lm_head.t()).float()
        return tp_all_gather(lg, dim=-1, ctx=self.p)
