"""Operator layer: GPU tensors run the hand-written gfx950 HIP kernels of ``nv_genai_amd._C``;
CPU tensors run the fp32 PyTorch references in :mod:`nv_genai_amd.ops.reference`.

There is no silent fallback on the GPU: if the extension is missing or fails to load, every
GPU call raises (so a GPU test can never pass on an eager-PyTorch substitute).
"""
from __future__ import annotations

import contextlib

from typing import Optional, Tuple

import torch

from . import reference as ref
from . import skinny
from .skinny import PartialSum

_C = None
_C_ERR: Optional[BaseException] = None
try:  # pragma: no cover - depends on the built artefact
    from .. import _C as _C  # type: ignore
except BaseException as e:  # noqa: BLE001
    _C_ERR = e


def kernels():
    """The loaded HIP extension; raises loudly when it is unavailable."""
    if _C is None:
        raise RuntimeError(
            "nv_genai_amd._C (gfx950 HIP kernels) is not loadable: "
            f"{_C_ERR!r}. Build it with `python -m nv_genai_amd._build`.")
    return _C


def have_kernels() -> bool:
    return _C is not None


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


# ------------------------------------------------------------------------- norms
def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, out: Optional[torch.Tensor] = None):
    if not _gpu(x):
        r = ref.rmsnorm(x, w, eps)
        if out is not None:
            out.copy_(r)
            return out
        return r
    if out is None:
        out = torch.empty(x.shape, dtype=x.dtype, device=x.device)
    kernels().rmsnorm(out, x, w, float(eps))
    return out


def add_rmsnorm(resid: torch.Tensor, delta: torch.Tensor, w: torch.Tensor, eps: float,
                out: Optional[torch.Tensor] = None):
    """resid += delta (in place); returns rmsnorm(resid) * w."""
    if not _gpu(resid):
        r = ref.add_rmsnorm(resid, delta, w, eps)
        if out is not None:
            out.copy_(r)
            return out
        return r
    if out is None:
        out = torch.empty_like(resid)
    kernels().add_rmsnorm(out, resid, delta, w, float(eps))
    return out


def layernorm(x, g, b, eps, resid=None, out=None):
    if not _gpu(x):
        return ref.layernorm(x, g, b, eps, resid)
    if out is None:
        out = torch.empty_like(x)
    kernels().layernorm(out, x, resid, g, b, float(eps))
    return out


def add_layernorm(resid, delta, g, b, eps, out=None):
    """resid += delta (in place); returns LayerNorm(resid) * g + b."""
    if not _gpu(resid):
        r = ref.add_layernorm(resid, delta, g, b, eps)
        if out is not None:
            out.copy_(r)
            return out
        return r
    if out is None:
        out = torch.empty_like(resid)
    kernels().add_layernorm(out, resid, delta, g, b, float(eps))
    return out


def gelu_tanh_mul(x: torch.Tensor, out: Optional[torch.Tensor] = None):
    """GeGLU: [T, 2F] = [gate | up] -> gelu_tanh(gate) * up [T, F]."""
    if not _gpu(x):
        return ref.gelu_tanh_mul(x)
    if out is None:
        out = torch.empty(x.shape[0], x.shape[1] // 2, dtype=x.dtype, device=x.device)
    kernels().gelu_tanh_mul(out, x)
    return out


def check_gemm_weight(w: torch.Tensor, what: str = "weight") -> torch.Tensor:
    """Library-GEMM operand guard: a weight must be a plain row-major matrix (2-D, unit column
    stride, row stride >= its width, 16-B aligned). The round-3 small-M probe faulted the GPU
    (hipErrorIllegalAddress) inside the library's batched split-K GEMM when it was handed a
    permuted [s, K/s, N] view of a weight (the batch dimension carved out of K, so each batch's
    rows are strided views into the transposed matrix); such views are rejected here instead of
    reaching the library. Returns ``w``."""
    if w.dim() != 2 or w.stride(1) != 1 or w.stride(0) < w.shape[1] or w.data_ptr() % 16:
        raise ValueError(f"{what}: the GEMM takes a contiguous row-major [N, K] matrix, got shape "
                         f"{tuple(w.shape)} strides {tuple(w.stride())}; make it .contiguous() once at load")
    return w


def linear(x: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``x @ w^T`` on the library GEMM with the operand guard (:func:`check_gemm_weight`)."""
    check_gemm_weight(w)
    if x.dim() != 2 or x.stride(1) != 1:
        x = x.contiguous()
    return torch.matmul(x, w.t(), out=out) if out is not None else x @ w.t()


def linear_rows_split(x: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None,
                      split: int = 0) -> torch.Tensor:
    """``x @ w^T`` (library GEMM) with the rows cut at ``split`` when ``x`` has more: the first
    ``split`` rows, then the rest, into disjoint row ranges of one output. At N = 4,096 a
    4,352-row GEMM is 272 output tiles of 256 x 256 — one full wave on 256 CUs plus a 16-tile
    second wave — while 4,096 rows are exactly one wave and the 256-row remainder runs right
    after on MALL-warm weights (benchmarks/row_split_gemm.py)."""
    M = x.shape[0]
    check_gemm_weight(w)
    if out is None:
        out = torch.empty(M, w.shape[0], dtype=x.dtype, device=x.device)
    if split <= 0 or M <= split:
        return torch.matmul(x, w.t(), out=out)
    torch.matmul(x[:split], w.t(), out=out[:split])
    torch.matmul(x[split:], w.t(), out=out[split:])
    return out


def pack_weight(w: torch.Tensor, BN: int, epi: int = 0) -> torch.Tensor:
    """Tile-packed image of an nn.Linear weight [N, K] for the skinny GEMM with a BN-row block:
    [nN * K/64 * BN, 64] where tile (block nb, K step kt) holds the block's BN weight rows of
    columns [64 kt, 64 kt + 64) contiguously — the order the kernel streams them. SwiGLU
    (``epi`` 2, w = [gate | up]): each block's rows are [gate f..f+15 | up f..f+15] per 32-row
    group of each wave's range, as the kernel reads them. A ragged last block repeats row N-1."""
    N, K = w.shape
    if epi == 2:
        F = N // 2
        nN = F // (BN // 2)
        r = torch.arange(BN)
        # the kernel's 2x2 / 4-wave layouts split BN over WN waves; the gate/up interleave is per
        # 32-row group within a wave's RW rows, which for every WN equals per 32-row group of BN
        f = (r >> 5) * 16 + (r & 15)
        up = (r >> 4) & 1
        rows = torch.stack([nb * (BN // 2) + f + up * F for nb in range(nN)])
    else:
        nN = -(-N // BN)
        rows = (torch.arange(nN * BN).clamp_max(N - 1)).view(nN, BN)
    nk = K // 64
    g = w.index_select(0, rows.reshape(-1).to(w.device)).view(nN, BN, nk, 64)
    return g.permute(0, 2, 1, 3).contiguous().view(nN * nk * BN, 64)


def pack_rows(x: torch.Tensor, BM: int) -> torch.Tensor:
    """Tile-packed image of activation rows x [M, K] for a BM-row token tile: [nM * K/64 * BM, 64]
    (rows past M zero)."""
    M, K = x.shape
    nM = -(-M // BM)
    xp = torch.zeros(nM * BM, K, dtype=x.dtype, device=x.device)
    xp[:M] = x
    return xp.view(nM, BM, K // 64, 64).permute(0, 2, 1, 3).contiguous().view(-1, 64)


def skinny_gemm(x: torch.Tensor, w: torch.Tensor, cfg: int, split: int = 1, epi: int = 0,
                out: Optional[torch.Tensor] = None, krot: int = 0, n_out: int = 0,
                x_rows: int = 0, k_in: int = 0) -> torch.Tensor:
    """Decode-shape projection GEMM (gemm_skinny.hip) with an explicit tile configuration:
    ``epi`` 0 -> bf16 ``x @ w^T``; 1 -> fp32 partial slabs [split, M, N] (K split ``split`` ways);
    2 -> SwiGLU ``silu(x @ w[:F]^T) * (x @ w[F:]^T)`` [M, F]. CPU tensors: the fp32 reference.
    ``n_out`` > 0: ``w`` is the :func:`pack_weight` image for this cfg and ``n_out`` the output
    features (N, or F for SwiGLU). ``x_rows`` > 0: ``x`` is the :func:`pack_rows` image for
    this cfg, ``x_rows`` its token rows and ``k_in`` its K."""
    M = x_rows or x.shape[0]
    if n_out and not _gpu(x):
        raise ValueError("packed skinny weights are a GPU layout")
    if not _gpu(x):
        y = x.float() @ w.float().t()
        if epi == 2:
            F = w.shape[0] // 2
            return (torch.nn.functional.silu(y[:, :F]) * y[:, F:]).to(x.dtype)
        if epi == 1:   # one slab holding the whole sum, the rest zero
            p = torch.zeros(split, M, w.shape[0])
            p[0] = y
            return p
        return y.to(x.dtype)
    N = n_out if n_out else (w.shape[0] // 2 if epi == 2 else w.shape[0])
    if out is None:
        out = (torch.empty(split, M, N, dtype=torch.float32, device=x.device) if epi == 1
               else torch.empty(M, N, dtype=x.dtype, device=x.device))
    kernels().skinny_gemm(out, x, w, int(epi), int(split), int(cfg), int(krot), 1 if n_out else 0, int(n_out),
                          int(x_rows), int(k_in))
    return out


GEMV_MAX_M = 4


def gemv(x: torch.Tensor, w: torch.Tensor, epi: int = 0, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Weight-streaming GEMV for M <= 4 token rows (gemv.hip): ``epi`` 0 -> bf16 ``x @ w^T``,
    1 -> fp32 ``x @ w^T`` (LM-head logits), 2 -> SwiGLU ``silu(x @ w[:F]^T) * (x @ w[F:]^T)``.
    CPU tensors: the fp32 reference."""
    if not _gpu(x):
        y = x.float() @ w.float().t()
        if epi == 2:
            F = w.shape[0] // 2
            return (torch.nn.functional.silu(y[:, :F]) * y[:, F:]).to(x.dtype)
        return y if epi == 1 else y.to(x.dtype)
    M = x.shape[0]
    N = w.shape[0] // 2 if epi == 2 else w.shape[0]
    if out is None:
        out = torch.empty(M, N, dtype=torch.float32 if epi == 1 else x.dtype, device=x.device)
    kernels().gemv(out, x, w, int(epi))
    return out


def splitk_reduce(P: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bf16 sum of the K-split partial slabs P [S, M, N]."""
    S, M, N = P.shape
    if not _gpu(P):
        return P.sum(0).to(torch.bfloat16)
    if out is None:
        out = torch.empty(M, N, dtype=torch.bfloat16, device=P.device)
    kernels().splitk_reduce(out, P, int(S))
    return out


def splitk_swiglu(P: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """silu(gate) * up of a K-split gate / up projection: P [S, M, 2F] fp32 partial slabs in the
    standard [gate | up] column order -> bf16 [M, F]."""
    S, M, N2 = P.shape
    F = N2 // 2
    if not _gpu(P):
        s = P.float().sum(0)
        return (torch.nn.functional.silu(s[:, :F]) * s[:, F:]).to(torch.bfloat16)
    if out is None:
        out = torch.empty(M, F, dtype=torch.bfloat16, device=P.device)
    kernels().splitk_swiglu(out, P, int(S))
    return out


def splitk_add_rmsnorm(resid: torch.Tensor, P: torch.Tensor, w: torch.Tensor, eps: float,
                       out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """resid += sum of the partial slabs P [S, M, H] (in place, one bf16 rounding); returns
    rmsnorm(resid) * w."""
    if not _gpu(resid):
        s = (resid.float() + P.float().sum(0)).to(resid.dtype)
        resid.copy_(s)
        r = ref.rmsnorm(resid, w, eps)
        if out is not None:
            out.copy_(r)
            return out
        return r
    if out is None:
        out = torch.empty_like(resid)
    kernels().splitk_add_rmsnorm(out, resid, P, int(P.shape[0]), w, float(eps))
    return out


def silu_mul(x: torch.Tensor, out: Optional[torch.Tensor] = None):
    if not _gpu(x):
        return ref.silu_mul(x)
    if out is None:
        out = torch.empty(x.shape[0], x.shape[1] // 2, dtype=x.dtype, device=x.device)
    kernels().silu_mul(out, x)
    return out


_GELU_MODES = {False: 0, "none": 0, True: 1, "tanh": 1, "quick": 2}


def bias_gelu_(x: torch.Tensor, bias: Optional[torch.Tensor], approximate=False):
    """x = gelu(x + bias) in place; ``approximate``: False / "none" (erf), True / "tanh"
    (StarCoder2, Gemma) or "quick" (CLIP's x * sigmoid(1.702 x))."""
    if not _gpu(x):
        return ref.bias_gelu_(x, bias, approximate)
    kernels().bias_gelu(x, bias, _GELU_MODES[approximate])
    return x


# ------------------------------------------------------------------------- rope / kv
def rope_cache_(qkv, pos, cos_sin, slots, kc, vc, Hq: int, Hkv: int, D: int,
                kv_scales=(1.0, 1.0), partial: Optional[PartialSum] = None):
    """RoPE on q / k in place + paged KV write. The caches are bf16, or fp8 e4m3fn holding
    k / kv_scales[0] and v / kv_scales[1]. ``partial``: the projection came as K-split fp32
    slabs; the kernel sums them and fills ``qkv`` (then output only) with the rotated q / k and
    the v columns."""
    if partial is not None and not _gpu(qkv):
        qkv.copy_(partial.slabs.sum(0).to(qkv.dtype))
        partial = None
    if not _gpu(qkv):
        return ref.rope_cache_(qkv, pos, cos_sin, slots, kc, vc, Hq, Hkv, D, kv_scales)
    kernels().rope_cache(qkv, pos, cos_sin, slots, kc, vc, Hq, Hkv, D, float(kv_scales[0]),
                         float(kv_scales[1]), None if partial is None else partial.slabs)
    return qkv


# ------------------------------------------------------------------------- attention
class DecodeWorkspace:
    """Split-K partition buffers for decode attention, sized for (max_seqs, Hq, max_ctx).

    The number of key partitions per (sequence, kv head) adapts to the batch: none once the
    batch alone gives >= 4 workgroups per CU (at 256 x 1400-token sequences one partition
    reads the KV stream 9 % faster than 16-page partitions and needs no combine kernel,
    benchmarks/kernel_bench.py), otherwise enough to reach ~2048 workgroups. The kernel
    divides each sequence's own pages evenly over the partitions, so the split also works
    for hipGraphs captured with the worst-case context. ``pages_per_part`` fixes the split
    (partitions = pages(max_ctx) / pages_per_part) instead."""

    TARGET_WGS = 2048
    FILL_WGS = 1024
    MAX_PARTS = 16
    DMA_WGS = 256      # LDS-DMA kernel (bf16, head_dim 128): one workgroup per CU

    def __init__(self, max_seqs: int, Hq: int, Hkv: int, max_ctx: int, device,
                 pages_per_part: Optional[int] = None, D: int = 128, kv_fp8: bool = False):
        self.pages = (max_ctx + 63) // 64
        self.fixed = pages_per_part
        self.Hkv = Hkv
        self.max_ctx = max_ctx
        self.dma = D == 128 and not kv_fp8
        need = max(b * self.nparts(b) for b in range(1, max_seqs + 1))
        self.ml = torch.empty(need * Hq * 2, dtype=torch.float32, device=device)
        self.o = torch.empty(need * Hq * D, dtype=torch.float32, device=device)
        self.D = D

    def nparts(self, B: int) -> int:
        if self.fixed:
            return -(-self.pages // max(1, self.fixed))
        items = B * self.Hkv
        if self.dma:
            # ~one busy workgroup per CU (the kernel gives every wave >= 1 page, so short
            # contexts use fewer partitions than this; graph replay, kernel_bench decode_small)
            return max(1, min(-(-self.DMA_WGS // items), self.MAX_PARTS))
        if items >= self.FILL_WGS:
            return 1
        return max(1, min(-(-self.TARGET_WGS // items), self.MAX_PARTS, max(1, self.pages // 4)))

    def pages_per_part(self, B: int, max_ctx: Optional[int] = None) -> int:
        """Grid sizing for the launcher: ceil(pages(max_ctx) / nparts)."""
        pages = (int(max_ctx if max_ctx is not None else self.max_ctx) + 63) // 64
        return max(1, -(-pages // self.nparts(B)))


KERNEL_FORMS = ("decode_dma", "decode_nt", "search_dma", "prefill_v1", "prefill_ks", "rope_vnt",
                "decode_dma_aux")


def kernel_form(name: str) -> int:
    """Current value of an A/B kernel form (csrc/kernels/kernels.h KernelForm; starts from its
    NGA_* environment variable, read once)."""
    return int(kernels().kernel_form(name))


@contextlib.contextmanager
def kernel_forms(**forms):
    """Select kernel forms for a block and restore them after, e.g.
    ``with ops.kernel_forms(decode_dma=2): ...`` (tests and A/B benchmarks; a hipGraph keeps the
    form it was captured with)."""
    C = kernels()
    old = {k: int(C.kernel_form(k)) for k in forms}
    try:
        for k, v in forms.items():
            C.set_kernel_form(k, int(v))
        yield
    finally:
        for k, v in old.items():
            C.set_kernel_form(k, v)


def decode_attention(q, kc, vc, block_tables, ctx_lens, Hq, Hkv, max_ctx, scale,
                     out=None, ws: Optional[DecodeWorkspace] = None, window: int = 0,
                     kv_scales=(1.0, 1.0), skip_empty: bool = False):
    """Paged GQA decode attention (head_dim 128 or 256); ``window`` > 0: sliding window;
    bf16 or fp8 e4m3fn caches (``kv_scales`` = the fp8 caches' K / V scales). ``skip_empty``:
    rows with ctx_len 0 are left untouched (not zeroed) — a graph-captured launch over a
    bucket of rows of which only the first few are this step's decode rows."""
    D = kc.shape[3]
    if not _gpu(q):
        r = ref.decode_attention(q, kc, vc, block_tables, ctx_lens, Hq, Hkv, scale, D=D,
                                 window=window, kv_scales=kv_scales)
        if out is not None:
            if skip_empty:
                live = ctx_lens[: r.shape[0]] > 0
                out[: r.shape[0], : r.shape[1]][live] = r[live].to(out.dtype)
            else:
                out[: r.shape[0], : r.shape[1]].copy_(r)
            return out
        return r
    B = ctx_lens.numel()
    if out is None:
        out = torch.empty(B, Hq * D, dtype=q.dtype, device=q.device)
    if ws is None:
        ws = DecodeWorkspace(B, Hq, Hkv, max_ctx, q.device, D=D, kv_fp8=kc.dtype != torch.bfloat16)
    assert max_ctx <= ws.max_ctx and ws.D == D
    kernels().decode_attention(out, q, kc, vc, block_tables, ctx_lens, Hq, Hkv, int(max_ctx),
                               float(scale), ws.pages_per_part(B, max_ctx), ws.ml, ws.o,
                               int(window), float(kv_scales[0]), float(kv_scales[1]), bool(skip_empty))
    return out


def prefill_attention_paged(q, kc, vc, block_tables, cu_q, ctx_lens, Hq, Hkv, D, max_q_len,
                            scale, out=None, causal=True, window: int = 0, impl: int = 0,
                            kv_scales=(1.0, 1.0)):
    """Paged prefill attention. ``impl``: 0 picks the kernel by problem size, 1 forces the
    16x16-MFMA kernel, 2 the 32x32-MFMA kernel (head_dim 128, bf16 caches), 3 its 8-wave
    split-key form (few prompts: two wave groups walk alternate key tiles of the same row
    block and merge in LDS) — for tests and A/B runs; 4 picks by size for a prefill that
    runs alone (no decode attention beside it: the 32x32 kernel from one prompt up, the
    split-key form for ~one row block per CU). fp8 e4m3fn caches (``kv_scales``) run the
    16x16 kernel."""
    if not _gpu(q):
        r = ref.prefill_attention_paged(q, kc, vc, block_tables, cu_q, ctx_lens, Hq, Hkv, D,
                                        scale, causal, window, kv_scales)
        if out is not None:
            out[:, : r.shape[1]].copy_(r)
            return out
        return r
    if out is None:
        out = torch.empty(q.shape[0], Hq * D, dtype=q.dtype, device=q.device)
    kernels().prefill_attention(out, q, None, None, kc, vc, block_tables, cu_q, ctx_lens, Hq,
                                Hkv, D, int(max_q_len), float(scale), bool(causal), int(window),
                                int(impl), float(kv_scales[0]), float(kv_scales[1]))
    return out


def prefill_rows_per_block(Hq: int, Hkv: int) -> int:
    """Query rows of one row block of the 32x32 prefill kernel (4 waves = 4 heads x 32 rows,
    2 heads x 2 x 32, or 1 head x 4 x 32 by the GQA group size)."""
    G = Hq // Hkv
    hpw = 4 if G % 4 == 0 else 2 if G % 2 == 0 else 1
    return 32 * (4 // hpw)


def plan_prefill_items(cu, ctx, first: int, n: int, Hq: int, Hkv: int, window: int = 0,
                       out: Optional["np.ndarray"] = None, rw: Optional[int] = None):
    """Host work list of the work-list prefill kernel for sequences [first, n) of a step
    (numpy ``cu`` [n+1] token offsets, ``ctx`` [n] context lengths): one (sequence, row
    block) pair per row block, longest causal key range first (so the fixed grid's
    workgroups take the long blocks first). Returns an int32 [k, 2] array (written into
    ``out`` when given). ``rw``: rows per block (default: the 32x32 kernel's; 64 for the
    16x16 kernel's tiles)."""
    import numpy as np

    rw = rw or prefill_rows_per_block(Hq, Hkv)
    cu = np.asarray(cu[first: n + 1], dtype=np.int64)
    ql = cu[1:] - cu[:-1]
    cx = np.asarray(ctx[first:n], dtype=np.int64)
    nb = (ql + rw - 1) // rw
    seq = np.repeat(np.arange(first, n, dtype=np.int64), nb)
    starts = np.repeat(np.cumsum(nb) - nb, nb)
    qb = np.arange(int(nb.sum()), dtype=np.int64) - starts
    qls, cxs = ql[seq - first], cx[seq - first]
    last = cxs - qls + np.minimum(qls - 1, qb * rw + rw - 1)      # last visible key of the block
    first_key = np.maximum(0, cxs - qls + qb * rw - window + 1) if window > 0 else np.zeros_like(last)
    tiles = last // 64 + 1 - first_key // 64
    order = np.argsort(-tiles, kind="stable")
    k = len(order)
    res = out[:k] if out is not None else np.empty((k, 2), dtype=np.int32)
    res[:, 0] = seq[order]
    res[:, 1] = qb[order]
    return res


def worklist_rows(impl: int, Hq: int, Hkv: int) -> int:
    """Query rows per work item: the 32x32 kernel's row block (impl 2) or the 16x16
    kernel's 64-row tile (impl 1)."""
    return prefill_rows_per_block(Hq, Hkv) if impl == 2 else 64


def prefill_attention_worklist(q, kc, vc, block_tables, cu_q, ctx_lens, Hq, Hkv, scale,
                               items, n_items, grid: int = 512, ks: int = 1, out=None,
                               causal: bool = True, window: int = 0, impl: int = 2,
                               kv_scales=(1.0, 1.0)):
    """Paged prefill attention driven by a device work list (``plan_prefill_items`` with
    ``rw = worklist_rows(impl, ...)``): rows are absolute token rows of the step, ``items``
    [>=n, 2] int32 and ``n_items`` a 1-element int32 tensor on the device. The launch shape
    (``grid`` workgroups x ``ks`` wave groups) is fixed, so one hipGraph capture serves
    every step's list. Rows no item covers are left untouched. ``impl`` 2: the 32x32 kernel
    (bf16 head_dim-128 pages), 1: the 16x16 kernel (head_dim 64 / 128 / 256, bf16 or fp8
    pages with ``kv_scales``)."""
    D = kc.shape[3]
    if not _gpu(q):
        return ref.prefill_attention_worklist(q, kc, vc, block_tables, cu_q, ctx_lens, Hq, Hkv, scale,
                                              items, n_items, out, causal, window,
                                              worklist_rows(impl, Hq, Hkv), D, kv_scales)
    if out is None:
        out = torch.zeros(q.shape[0], Hq * D, dtype=q.dtype, device=q.device)
    kernels().prefill_attention_worklist(out, q, kc, vc, block_tables, cu_q, ctx_lens, int(Hq), int(Hkv),
                                         float(scale), bool(causal), int(window), items, n_items,
                                         int(grid), int(ks), int(impl), float(kv_scales[0]),
                                         float(kv_scales[1]))
    return out


def varlen_attention(q, k, v, cu, Hq, Hkv, D, max_len, scale, causal=False, out=None):
    """Packed variable-length attention (no paging): q/k/v rows share the cu offsets."""
    if not _gpu(q):
        return ref.varlen_attention(q, k, v, cu, Hq, Hkv, D, scale, causal)
    if out is None:
        out = torch.empty(q.shape[0], Hq * D, dtype=q.dtype, device=q.device)
    kernels().prefill_attention(out, q, k, v, None, None, None, cu, None, Hq, Hkv, D,
                                int(max_len), float(scale), bool(causal), 0, 0, 1.0, 1.0)
    return out


# ------------------------------------------------------------------------- MoE
MOE_BN = 128       # weight rows per grouped-GEMM tile


class MoEWorkspace:
    """Routing / permutation buffers of the grouped MoE GEMMs for up to ``rows`` tokens.

    A serving model owns one, sized once for its largest step before any hipGraph capture
    (``LlamaModel.moe_ws``, set by the engine) and passed to :func:`moe_ffn`, so two engines
    in one process never share routing buffers. Callers without one (benchmarks, tests) use
    the per-(device, top-k, experts) cache of :meth:`get`; a workspace it outgrows is retired,
    not freed, because a graph captured earlier may still write to its buffers."""

    _cache = {}
    _retired = []

    @classmethod
    def get(cls, rows: int, k: int, E: int, device):
        key = (str(device), k, E)
        ws = cls._cache.get(key)
        if ws is None or ws.rows < rows:
            if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
                raise RuntimeError("MoE workspace must be sized before graph capture")
            if ws is not None:
                cls._retired.append(ws)
            ws = cls(max(rows, 64), k, E, device)
            cls._cache[key] = ws
        return ws

    def __init__(self, rows: int, k: int, E: int, device):
        self.rows, self.k, self.E = rows, k, E
        M = rows * k
        self.mt_cap = max(1, -(-M // 64)) + E          # M-tile bound at BM = 64 (the larger)
        i32 = dict(dtype=torch.int32, device=device)
        self.ids = torch.empty(M, **i32)
        self.w = torch.empty(M, dtype=torch.float32, device=device)
        self.sorted_tok = torch.empty(M, **i32)
        self.sorted_w = torch.empty(M, dtype=torch.float32, device=device)
        self.inv = torch.empty(M, **i32)
        self.tiles = torch.empty(self.mt_cap * 3, **i32)


def moe_ffn(x: torch.Tensor, router: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, k: int,
            expert0: int = 0, act: str = "silu", ws: Optional["MoEWorkspace"] = None) -> torch.Tensor:
    """Sparse MoE MLP on rows x [T, H] -> [T, H] (a TP partial sum when the experts or their
    FFN dims are split over ranks). ``w13`` [E, 2F, H] = [gate | up] rows per local expert,
    ``w2`` [E, H, F]; the router [num_experts, H] scores every expert.

    GPU: router GEMM (hipBLASLt) -> ``moe_route`` (softmax top-k) -> ``moe_align`` (per-
    expert counts, sorted token order, M-tile table) -> gathered grouped MFMA GEMM with the
    activation fused in its epilogue (gate and up rows interleaved per 16-row MFMA tile) ->
    grouped down GEMM scaled by the routing weight -> ``moe_combine`` (top-k rows summed in
    fp32 per token)."""
    if not _gpu(x):
        return ref.moe_ffn(x, router, w13, w2, k, expert0, act)
    C = kernels()
    T, H = x.shape
    E, F2, K = w13.shape
    F = F2 // 2
    out = torch.empty(T, H, dtype=x.dtype, device=x.device)
    if T == 0:
        return out
    if ws is None:
        ws = MoEWorkspace.get(T, k, E, x.device)
    elif ws.rows < T or ws.k != k or ws.E != E:
        raise ValueError(f"MoE workspace for {ws.rows} rows / top-{ws.k} / {ws.E} experts cannot "
                         f"take {T} rows / top-{k} / {E} experts")
    M = T * k
    # 64-row M tiles while the experts average <= 4 of them (decode), 128 beyond (prefill)
    bm = 64 if M <= 256 * E else 128
    mt = -(-M // bm) + E                                           # M-tile bound of this call
    logits = x @ router.t()                                        # [T, num_experts] bf16
    C.moe_route(logits, int(k), ws.ids, ws.w)
    C.moe_align(ws.ids, ws.w, T, int(k), int(expert0), E, bm, ws.sorted_tok, ws.sorted_w, ws.inv,
                ws.tiles, mt)
    h = torch.empty(M, F, dtype=x.dtype, device=x.device)
    C.moe_gemm(x, w13, ws.sorted_tok, ws.sorted_w, ws.tiles, mt, bm, h, 0,
               0 if act == "silu" else 1)
    y = torch.empty(M, H, dtype=x.dtype, device=x.device)
    C.moe_gemm(h, w2, ws.sorted_tok, ws.sorted_w, ws.tiles, mt, bm, y, 1, 0)
    C.moe_combine(y, ws.inv, T, int(k), out)
    return out


# ------------------------------------------------------------------------- sampling
def sample(logits, temperature, top_k, top_p, seeds, steps, rep_penalty=None, history=None,
           out_tok=None, out_lp=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Sample one token per row. ``logits`` (fp32, [B, V]) may be modified in place."""
    if not _gpu(logits):
        return ref.sample(logits, temperature, top_k, top_p, seeds, steps, rep_penalty, history)
    B = logits.shape[0]
    if out_tok is None:
        out_tok = torch.empty(B, dtype=torch.int32, device=logits.device)
    if out_lp is None:
        out_lp = torch.empty(B, dtype=torch.float32, device=logits.device)
    kernels().sample(logits, temperature, top_k, top_p, rep_penalty, history, seeds, steps,
                     out_tok, out_lp)
    return out_tok, out_lp


# ------------------------------------------------------------------------- FP8 W8A8
FP8 = torch.float8_e4m3fn
FP8_MAX = 448.0


def quant_fp8_rows(x: torch.Tensor, mode: int = 0, pad_to: int = 16):
    """Row-wise FP8 quantisation of a GEMM input: mode 0 quantises x [M, H]; mode 1 the
    SwiGLU of x [M, 2F] = [gate | up]. Returns (y [Mp, H] e4m3fn, scale [Mp, 1] fp32) with M
    padded to ``pad_to`` rows (zero rows, scale 1) for the FP8 GEMM's tile constraints."""
    M = x.shape[0]
    H = x.shape[1] if mode == 0 else x.shape[1] // 2
    Mp = -(-max(M, 1) // pad_to) * pad_to
    if not _gpu(x):
        return ref.quant_fp8_rows(x, mode, Mp)
    y = torch.empty(Mp, H, dtype=FP8, device=x.device)
    s = torch.empty(Mp, 1, dtype=torch.float32, device=x.device)
    if Mp > M:
        y[M:].view(torch.uint8).zero_()
        s[M:].fill_(1.0)
    kernels().quant_fp8_rows(x, int(mode), y, s)
    return y, s


def quantize_weight_fp8(w: torch.Tensor):
    """[N, K] -> (e4m3fn [N, K], per-output-channel scale [1, N] fp32)."""
    wf = w.float()
    s = wf.abs().amax(1, keepdim=True).clamp_min(1e-12) / FP8_MAX
    w8 = (wf / s).clamp(-FP8_MAX, FP8_MAX).to(FP8)
    return w8.contiguous(), s.t().contiguous()


def fp8_linear(x8: torch.Tensor, sx: torch.Tensor, w8: torch.Tensor, sw: torch.Tensor, M: int) -> torch.Tensor:
    """bf16 [M, N] = (x8 * sx) @ (w8 * sw^T)^T: a row-scaled hipBLASLt FP8 GEMM on the GPU."""
    if x8.is_cuda:
        y = torch._scaled_mm(x8, w8.t(), scale_a=sx, scale_b=sw, out_dtype=torch.bfloat16)
    else:
        y = ((x8.float() * sx) @ (w8.float() * sw.t()).t()).to(torch.bfloat16)
    return y[:M]


# ------------------------------------------------------------------------- vector search
def score(Q, X, row_bias=None, dot_scale: float = 1.0, out=None):
    if not _gpu(X):
        return ref.score(Q, X, row_bias, dot_scale)
    if out is None:
        out = torch.empty(Q.shape[0], X.shape[0], dtype=torch.float32, device=X.device)
    kernels().score(Q, X, row_bias, out, float(dot_scale))
    return out


TOPK_SEG = 4096


def topk(S: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Exact row-wise top-k (descending) of a fp32 score matrix: per-4096 segment select,
    then a merge select over the segment winners."""
    k = int(min(k, S.shape[1]))
    if not _gpu(S):
        return ref.topk(S, k)
    C = kernels()
    rows, n = S.shape
    nseg = (n + TOPK_SEG - 1) // TOPK_SEG
    v1 = torch.empty(rows, nseg * k, dtype=torch.float32, device=S.device)
    i1 = torch.empty(rows, nseg * k, dtype=torch.int64, device=S.device)
    C.topk(S, None, TOPK_SEG, k, v1, i1)
    if nseg == 1:
        return v1, i1
    v2 = torch.empty(rows, k, dtype=torch.float32, device=S.device)
    i2 = torch.empty(rows, k, dtype=torch.int64, device=S.device)
    C.topk(v1, i1, nseg * k, k, v2, i2)
    return v2, i2


def score_topk_blocks(nrows: int, rows_per_item: int, n_active_items: int, q_per_item: int,
                      dma: bool = False, cus: int = 256) -> int:
    """Blocks per work item of the fused score + top-k kernel: ~1024 resident blocks over the
    chip (512 for 64-query items, whose 8-wave blocks hold 128 KiB of query tile each), no
    more than the item's row tiles. The LDS-DMA form (``dma``, <= 16 queries per item) fills
    a CU's LDS with one block, so it gets one block per CU."""
    rows_per_tile = 256 if q_per_item > 32 else 128
    tiles = max(1, -(-rows_per_item // rows_per_tile))
    if dma:
        target = cus // max(1, n_active_items)
    else:
        target = (512 if q_per_item > 32 else 1024) // max(1, n_active_items)
    return int(max(1, min(tiles, max(4, target), 65535)))


_CUS = {}


def _cu_count(dev) -> int:
    d = torch.device(dev)
    if d not in _CUS:
        _CUS[d] = torch.cuda.get_device_properties(d).multi_processor_count
    return _CUS[d]


def search_topk(Q: torch.Tensor, X: torch.Tensor, row_bias=None, dot_scale: float = 1.0, k: int = 4):
    """Exact top-k rows of X [N, D] for every query of Q [nq, D] by S = dot_scale Q.X^T +
    row_bias, without materialising S: the fused MFMA score + per-block top-k kernel writes
    [nq, blocks, k] candidates and one ``topk`` pass merges them (K13: per-tile top-k fused
    into scoring, then the k-merge). Returns (scores [nq, k], rows [nq, k]; -inf / -1 where X
    has fewer than k live rows). Falls back to the score matrix + ``topk`` when k exceeds the
    kernel's register lists."""
    k = int(min(k, X.shape[0]))
    nq = Q.shape[0]
    if not _gpu(X):
        return ref.topk(ref.score(Q, X, row_bias, dot_scale), k)
    C = kernels()
    qpi = min(nq, 64)
    if k > C.score_topk_kmax(qpi) or nq == 0:
        return topk(score(Q, X, row_bias, dot_scale), k)
    items = -(-nq // 64)
    dma = bool(C.score_topk_dma_ok(X.shape[1], qpi))
    nblk = score_topk_blocks(X.shape[0], X.shape[0], items, qpi, dma, _cu_count(X.device) if dma else 256)
    cv = torch.empty(items * 64, nblk, k, dtype=torch.float32, device=X.device)
    cr = torch.empty(items * 64, nblk, k, dtype=torch.int64, device=X.device)
    C.score_topk(Q, X, row_bias, float(dot_scale), None, None, None, None, items, qpi, nblk, k, cv, cr)
    cv, cr = cv[:nq].view(nq, nblk * k), cr[:nq].view(nq, nblk * k)
    if nblk == 1:
        return cv, cr
    v = torch.empty(nq, k, dtype=torch.float32, device=X.device)
    r = torch.empty(nq, k, dtype=torch.int64, device=X.device)
    C.topk(cv, cr, nblk * k, k, v, r)
    return v, r


IVF_MAX_ITEMS = 65535   # score_topk's work-item limit (grid dimension)


def ivf_search_topk(Q: torch.Tensor, X: torch.Tensor, row_bias, dot_scale: float, probes: torch.Tensor,
                    list_beg: torch.Tensor, list_end: torch.Tensor, max_list_rows: int, k: int):
    """IVF list scan (K14) for a batch of queries in one launch: the (query, probe) pairs are
    grouped by list on the device (no host sync), every probed list is streamed once for all
    the queries that probe it by the fused score + top-k kernel, and each query's nprobe x
    blocks x k candidates are merged by one ``topk`` pass. ``probes`` [nq, nprobe] int64 list
    ids; ``list_beg`` / ``list_end`` [nlist] int64 row ranges of the list-sorted slab X.
    Returns (scores [nq, k], slab rows [nq, k]). Launches: plan (1 block), scan, k-merge."""
    nq, nprobe = probes.shape
    nlist = list_beg.numel()
    dev = X.device
    if not _gpu(X):
        return ref.ivf_search_topk(Q, X, row_bias, dot_scale, probes, list_beg, list_end, k)
    C = kernels()
    qpi = min(nq, 64)
    if nlist > 16384:    # the plan kernel's LDS list counters (IVF_PLAN_MAX_LISTS)
        return ref.ivf_search_topk(Q, X, row_bias, dot_scale, probes, list_beg, list_end, k)
    if k > C.score_topk_kmax(qpi):
        raise ValueError(f"IVF search: k={k} above the fused kernel's limit {C.score_topk_kmax(qpi)}")
    chunks = -(-nq // 64)
    n_items = nlist * chunks
    max_q = 64 * (IVF_MAX_ITEMS // nlist)
    if n_items > IVF_MAX_ITEMS:
        # the scan launch takes at most 65,535 (list, 64-query chunk) items: run the queries
        # in sub-batches that fit (nlist 4,096: 1,024 queries per launch)
        parts = [ivf_search_topk(Q[i:i + max_q], X, row_bias, dot_scale, probes[i:i + max_q], list_beg,
                                 list_end, max_list_rows, k) for i in range(0, nq, max_q)]
        return torch.cat([p[0] for p in parts]), torch.cat([p[1] for p in parts])
    probes = probes.to(torch.int64).contiguous()
    # one block groups the pairs by list: slot -> query, slot -> pair (candidate row)
    qtab = torch.empty(n_items * 64, dtype=torch.int32, device=dev)
    slot_rows = torch.empty(n_items * 64, dtype=torch.int32, device=dev)
    C.ivf_plan(probes, nlist, qtab, slot_rows)
    rb = list_beg if chunks == 1 else list_beg.repeat_interleave(chunks)
    re = list_end if chunks == 1 else list_end.repeat_interleave(chunks)
    dma = bool(C.score_topk_dma_ok(X.shape[1], qpi))
    nblk = score_topk_blocks(X.shape[0], max_list_rows, min(nlist, nq * nprobe), qpi, dma,
                             _cu_count(dev) if dma else 256)
    # candidates in (query, probe) order: [nq, nprobe * nblk * k] with no gather
    gv = torch.empty(nq * nprobe, nblk, k, dtype=torch.float32, device=dev)
    gr = torch.empty(nq * nprobe, nblk, k, dtype=torch.int64, device=dev)
    C.score_topk(Q, X, row_bias, float(dot_scale), rb, re, qtab, slot_rows, n_items, qpi, nblk, k, gv, gr)
    gv, gr = gv.view(nq, nprobe * nblk * k), gr.view(nq, nprobe * nblk * k)
    v = torch.empty(nq, k, dtype=torch.float32, device=dev)
    r = torch.empty(nq, k, dtype=torch.int64, device=dev)
    C.topk(gv, gr, gv.shape[1], k, v, r)
    return v, r


def embedding(ids: torch.Tensor, table: torch.Tensor, vocab_lo: int = 0, scale: float = 1.0, out=None):
    """Token rows of ``table`` (this rank's vocabulary shard starting at ``vocab_lo``; ids
    outside it give zero rows), times ``scale`` in bf16 (K8). GPU: the embedding.hip gather."""
    if not _gpu(table):
        return ref.embedding(ids, table, vocab_lo, scale)
    ids = ids.to(torch.int32).contiguous()
    if out is None:
        out = torch.empty(ids.numel(), table.shape[1], dtype=table.dtype, device=table.device)
    kernels().embedding(out, table, ids, int(vocab_lo), float(scale))
    return out


def pool_l2norm(hidden, cu, mode: int = 0, normalize: bool = True, out=None):
    if not _gpu(hidden):
        return ref.pool_l2norm(hidden, cu, mode, normalize)
    B = cu.numel() - 1
    if out is None:
        out = torch.empty(B, hidden.shape[1], dtype=torch.float32, device=hidden.device)
    kernels().pool_l2norm(hidden, cu, int(mode), bool(normalize), out)
    return out


_MARKER_SINK = {}


def region_marker(device, end: bool) -> None:
    """Launch the begin (``end=False``) or end marker kernel on ``device``'s current stream:
    a kernel trace (rocprofv3 --kernel-trace) then shows where a region such as bench.py's timed
    window starts and ends on the GPU timeline (scripts/summarize_prof.py uses them). No-op on
    the CPU."""
    device = torch.device(device)
    if device.type != "cuda":
        return
    sink = _MARKER_SINK.get(device)
    if sink is None:
        sink = _MARKER_SINK[device] = torch.zeros(1, dtype=torch.int32, device=device)
    kernels().region_marker(sink, 1 if end else 0)


def row_sqnorm(X, out=None):
    if not _gpu(X):
        return ref.row_sqnorm(X)
    if out is None:
        out = torch.empty(X.shape[0], dtype=torch.float32, device=X.device)
    kernels().row_sqnorm(X, out)
    return out


rope_cos_sin = ref.rope_cos_sin


# ---------------------------------------------------------------- DSP (FM-ASR front end)
def fir_c64(x: torch.Tensor, taps: torch.Tensor, hist: Optional[torch.Tensor] = None) -> torch.Tensor:
    if not _gpu(x):
        return ref.fir_c64(x, taps, hist)
    y = torch.empty_like(x)
    kernels().fir_c64(x, taps, hist, y)
    return y


def fm_demod(x: torch.Tensor, prev: Optional[complex] = None) -> torch.Tensor:
    if not _gpu(x):
        return ref.fm_demod(x, prev)
    n = x.numel() if prev is not None else max(0, x.numel() - 1)
    y = torch.empty(n, dtype=torch.float32, device=x.device)
    p = prev if prev is not None else 0j
    kernels().fm_demod(x, float(p.real), float(p.imag), prev is not None, y)
    return y


def resample_pcm(x: torch.Tensor, h: torch.Tensor, down: int, pre: int, nout: int, gain: float = 1.0):
    """-> (float32 samples, int16 PCM)."""
    if not _gpu(x):
        return ref.resample_pcm(x, h, down, pre, nout, gain)
    yf = torch.empty(nout, dtype=torch.float32, device=x.device)
    yi = torch.empty(nout, dtype=torch.int16, device=x.device)
    kernels().resample_pcm(x, h, int(down), int(pre), float(gain), yf, yi)
    return yf, yi
