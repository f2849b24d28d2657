"""Plain-PyTorch (fp32 math) reference implementations of every HIP kernel in
``nv_genai_amd/csrc/kernels``.

They serve two purposes: the numerics oracle of the kernel tests (a GPU kernel is compared
against the op below evaluated in fp32), and the CPU execution path used by the CPU-only
unit tests of the engine / chain server. Layouts and semantics match the kernels exactly:

* paged caches: K ``[num_blocks, Hkv, BS, D]``, V transposed ``[num_blocks, Hkv, D, BS]``;
* ``qkv`` is the fused projection output ``[T, (Hq + 2*Hkv) * D]``;
* sampling uses the same counter-based RNG (splitmix64 of ``seed + golden * (ctr + 1)``) and
  Gumbel-max draw, so CPU and GPU pick identical tokens for identical logits.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import numpy as np
import torch


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    r = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (xf * r * w.float()).to(x.dtype)


def add_rmsnorm(resid: torch.Tensor, delta: torch.Tensor, w: torch.Tensor, eps: float):
    s = (resid.float() + delta.float()).to(resid.dtype)
    resid.copy_(s)
    return rmsnorm(s, w, eps)


def layernorm(x, g, b, eps, resid=None):
    xf = x.float() + (resid.float() if resid is not None else 0.0)
    y = torch.nn.functional.layer_norm(xf, (x.shape[-1],), g.float(), b.float(), eps)
    return y.to(x.dtype)


def add_layernorm(resid, delta, g, b, eps):
    """resid += delta (stored in the residual dtype); returns LayerNorm(resid) * g + b."""
    s = (resid.float() + delta.float()).to(resid.dtype)
    resid.copy_(s)
    return layernorm(s, g, b, eps)


def gelu_tanh_mul(x: torch.Tensor) -> torch.Tensor:
    """GeGLU: x = [gate | up] -> gelu_tanh(gate) * up."""
    F = x.shape[-1] // 2
    g, u = x[..., :F].float(), x[..., F:].float()
    return (torch.nn.functional.gelu(g, approximate="tanh") * u).to(x.dtype)


def silu_mul(x: torch.Tensor) -> torch.Tensor:
    F = x.shape[-1] // 2
    g, u = x[..., :F].float(), x[..., F:].float()
    return (torch.nn.functional.silu(g) * u).to(x.dtype)


def bias_gelu_(x: torch.Tensor, bias: Optional[torch.Tensor], approximate=False) -> torch.Tensor:
    """approximate: False / "none" (erf GELU), True / "tanh", or "quick" (x * sigmoid(1.702 x))."""
    xf = x.float() + (bias.float() if bias is not None else 0.0)
    if approximate == "quick":
        y = xf * torch.sigmoid(1.702 * xf)
    else:
        y = torch.nn.functional.gelu(xf, approximate="tanh" if approximate in (True, "tanh") else "none")
    x.copy_(y.to(x.dtype))
    return x


def rope_cos_sin(max_pos: int, D: int, theta: float = 500000.0,
                 scaling: Optional[dict] = None) -> torch.Tensor:
    """[max_pos, D] fp32 table: cos of the D/2 frequencies, then sin (rotate-half layout).

    ``scaling`` implements Llama-3.1 style frequency scaling when given
    (factor, low_freq_factor, high_freq_factor, original_max_position_embeddings)."""
    inv = 1.0 / (theta ** (torch.arange(0, D, 2, dtype=torch.float64) / D))
    if scaling:
        factor = scaling.get("factor", 8.0)
        lo = scaling.get("low_freq_factor", 1.0)
        hi = scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        wavelen = 2 * math.pi / inv
        lo_wl, hi_wl = old / lo, old / hi
        smooth = (old / wavelen - lo) / (hi - lo)
        scaled = torch.where(wavelen > lo_wl, inv / factor, inv)
        mid = (wavelen <= lo_wl) & (wavelen >= hi_wl)
        scaled = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
        inv = scaled
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return torch.cat([f.cos(), f.sin()], dim=-1).float()


def _to_cache(x: torch.Tensor, cache: torch.Tensor, scale: float) -> torch.Tensor:
    """Cache element type: bf16 as is; fp8 e4m3fn stores x / scale, saturated to +-448."""
    if cache.dtype == torch.float8_e4m3fn:
        return (x.float() * (1.0 / scale)).clamp(-448.0, 448.0).to(cache.dtype)
    return x.to(cache.dtype)


def rope_cache_(qkv, pos, cos_sin, slots, kc, vc, Hq, Hkv, D, kv_scales=(1.0, 1.0)):
    T = qkv.shape[0]
    x = qkv.view(T, Hq + 2 * Hkv, D)
    cs = cos_sin[pos.long()]  # [T, D]
    c, s = cs[:, : D // 2].unsqueeze(1), cs[:, D // 2:].unsqueeze(1)
    rot = x[:, : Hq + Hkv].float()
    x1, x2 = rot[..., : D // 2], rot[..., D // 2:]
    out = torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1).to(qkv.dtype)
    x[:, : Hq + Hkv] = out
    if slots is not None:
        BS = kc.shape[2]
        sl = slots.long()
        ok = sl >= 0
        blk, off = sl[ok] // BS, sl[ok] % BS
        k = x[ok, Hq: Hq + Hkv]  # [n, Hkv, D]
        v = x[ok, Hq + Hkv:]
        kc[blk, :, off, :] = _to_cache(k, kc, kv_scales[0])
        vc[blk, :, :, off] = _to_cache(v, vc, kv_scales[1])
    return qkv


def _gather_kv(kc, vc, bt_row, ctx, kvh, kv_scales=(1.0, 1.0)):
    BS = kc.shape[2]
    n_pages = (ctx + BS - 1) // BS
    blocks = bt_row[:n_pages].long()
    k = kc[blocks, kvh].reshape(-1, kc.shape[3])[:ctx]  # [ctx, D]
    v = vc[blocks, kvh].permute(0, 2, 1).reshape(-1, vc.shape[2])[:ctx]
    if kc.dtype == torch.float8_e4m3fn:
        return k.float() * kv_scales[0], v.float() * kv_scales[1]
    return k.float(), v.float()


def decode_attention(q, kc, vc, block_tables, ctx_lens, Hq, Hkv, scale, D=128, window=0,
                     kv_scales=(1.0, 1.0)):
    """One query per sequence at position ctx - 1; ``window`` > 0 keeps only the last
    ``window`` keys (sliding-window attention: key j visible iff j > ctx - 1 - window)."""
    B = ctx_lens.numel()
    G = Hq // Hkv
    out = torch.zeros(B, Hq * D, dtype=q.dtype, device=q.device)
    for b in range(B):
        ctx = int(ctx_lens[b])
        if ctx == 0:
            continue
        lo = max(0, ctx - window) if window > 0 else 0
        for kvh in range(Hkv):
            k, v = _gather_kv(kc, vc, block_tables[b], ctx, kvh, kv_scales)
            k, v = k[lo:], v[lo:]
            qs = q[b, kvh * G * D:(kvh + 1) * G * D].view(G, D).float()
            p = torch.softmax(qs @ k.T * scale, dim=-1)
            out[b, kvh * G * D:(kvh + 1) * G * D] = (p @ v).reshape(-1).to(q.dtype)
    return out


def prefill_attention_paged(q, kc, vc, block_tables, cu_q, ctx_lens, Hq, Hkv, D, scale,
                            causal=True, window=0, kv_scales=(1.0, 1.0)):
    G = Hq // Hkv
    T = q.shape[0]
    out = torch.zeros(T, Hq * D, dtype=q.dtype, device=q.device)
    B = cu_q.numel() - 1
    for b in range(B):
        s0, s1 = int(cu_q[b]), int(cu_q[b + 1])
        ql, ctx = s1 - s0, int(ctx_lens[b])
        if ql == 0:
            continue
        qpos = torch.arange(ctx - ql, ctx, device=q.device)
        kpos = torch.arange(ctx, device=q.device)
        mask = kpos[None, :] <= qpos[:, None] if causal else torch.ones(ql, ctx, dtype=torch.bool, device=q.device)
        if window > 0:
            mask = mask & (kpos[None, :] > qpos[:, None] - window)
        for hq in range(Hq):
            k, v = _gather_kv(kc, vc, block_tables[b], ctx, hq // G, kv_scales)
            qs = q[s0:s1, hq * D:(hq + 1) * D].float()
            sc = (qs @ k.T) * scale
            sc = sc.masked_fill(~mask, float("-inf"))
            out[s0:s1, hq * D:(hq + 1) * D] = (torch.softmax(sc, -1) @ v).to(q.dtype)
    return out


def prefill_attention_worklist(q, kc, vc, block_tables, cu_q, ctx_lens, Hq, Hkv, scale, items, n_items,
                               out=None, causal=True, window=0, rw=128, D=128, kv_scales=(1.0, 1.0)):
    """The work-list kernel's semantics: every listed (sequence, row block) pair writes its
    RW query rows (absolute token rows cu_q[b] + RW qb ...) of every head; other rows of
    ``out`` are left as they are."""
    G = Hq // Hkv
    if out is None:
        out = torch.zeros(q.shape[0], Hq * D, dtype=q.dtype, device=q.device)
    n = int(n_items.reshape(-1)[0])
    for b, qb in items[:n].tolist():
        s0, s1 = int(cu_q[b]), int(cu_q[b + 1])
        ql, ctx = s1 - s0, int(ctx_lens[b])
        r0, r1 = qb * rw, min(ql, qb * rw + rw)
        if r0 >= r1:
            continue
        qpos = torch.arange(ctx - ql + r0, ctx - ql + r1, device=q.device)
        kpos = torch.arange(ctx, device=q.device)
        mask = kpos[None, :] <= qpos[:, None] if causal else torch.ones(r1 - r0, ctx, dtype=torch.bool,
                                                                        device=q.device)
        if window > 0:
            mask = mask & (kpos[None, :] > qpos[:, None] - window)
        for hq in range(Hq):
            k, v = _gather_kv(kc, vc, block_tables[b], ctx, hq // G, kv_scales)
            qs = q[s0 + r0:s0 + r1, hq * D:(hq + 1) * D].float()
            sc = ((qs @ k.T) * scale).masked_fill(~mask, float("-inf"))
            out[s0 + r0:s0 + r1, hq * D:(hq + 1) * D] = (torch.softmax(sc, -1) @ v).to(out.dtype)
    return out


def varlen_attention(q, k, v, cu, Hq, Hkv, D, scale, causal=False):
    G = Hq // Hkv
    T = q.shape[0]
    out = torch.zeros(T, Hq * D, dtype=q.dtype, device=q.device)
    for b in range(cu.numel() - 1):
        s0, s1 = int(cu[b]), int(cu[b + 1])
        n = s1 - s0
        if n == 0:
            continue
        for hq in range(Hq):
            kvh = hq // G
            qs = q[s0:s1, hq * D:(hq + 1) * D].float()
            ks = k[s0:s1, kvh * D:(kvh + 1) * D].float()
            vs = v[s0:s1, kvh * D:(kvh + 1) * D].float()
            sc = (qs @ ks.T) * scale
            if causal:
                m = torch.ones(n, n, dtype=torch.bool, device=q.device).tril()
                sc = sc.masked_fill(~m, float("-inf"))
            out[s0:s1, hq * D:(hq + 1) * D] = (torch.softmax(sc, -1) @ vs).to(q.dtype)
    return out


# ----------------------------------------------------------------------------- MoE
def moe_route(logits: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Mixtral routing: softmax over all experts (fp32), top-k, renormalised over the k.
    Returns (ids int32 [T, k], weights fp32 [T, k]) in descending-probability order."""
    p = torch.softmax(logits.float(), dim=-1)
    w, ids = torch.topk(p, k, dim=-1)
    w = w / w.sum(-1, keepdim=True)
    return ids.to(torch.int32), w


def moe_ffn(x, router, w13, w2, k, expert0=0, act="silu"):
    """Sparse MoE MLP of one layer on rows x [T, H] (fp32 math per expert):
    sum_j w_j * down_e(act(gate_e(x)) * up_e(x)) over the top-k experts e of each row that
    this rank holds (experts [expert0, expert0 + w13.shape[0]))."""
    logits = (x @ router.t())
    ids, wts = moe_route(logits, k)
    E, F2, _ = w13.shape
    F = F2 // 2
    out = torch.zeros(x.shape[0], w2.shape[1], dtype=torch.float32, device=x.device)
    for e in range(E):
        tok, slot = torch.where(ids == expert0 + e)
        if tok.numel() == 0:
            continue
        gu = x[tok].float() @ w13[e].float().t()
        g, u = gu[:, :F], gu[:, F:]
        h = (torch.nn.functional.silu(g) if act == "silu" else
             torch.nn.functional.gelu(g, approximate="tanh")) * u
        y = h.to(x.dtype).float() @ w2[e].float().t()
        out.index_add_(0, tok, y * wts[tok, slot].unsqueeze(1))
    return out.to(x.dtype)


# ----------------------------------------------------------------------------- sampling
_GOLD = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def hash_uniform(seed: int, ctr: np.ndarray) -> np.ndarray:
    """Same counter RNG as common.h::hash_uniform -> float32 in (0, 1]."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + _GOLD * (ctr.astype(np.uint64) + np.uint64(1))
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return ((z >> np.uint64(40)).astype(np.float32) + np.float32(1.0)) * np.float32(1.0 / 16777216.0)


def sample(logits, temperature, top_k, top_p, seeds, steps, rep_penalty=None, history=None):
    B, V = logits.shape
    x = logits.float().clone()
    toks = torch.zeros(B, dtype=torch.int32)
    lps = torch.zeros(B, dtype=torch.float32)
    for b in range(B):
        row = x[b]
        if rep_penalty is not None and history is not None and float(rep_penalty[b]) != 1.0:
            pen = float(rep_penalty[b])
            h = history[b].long()
            h = torch.unique(h[(h >= 0) & (h < V)])
            vals = row[h]
            row[h] = torch.where(vals > 0, vals / pen, vals * pen)
        t = float(temperature[b])
        k = int(top_k[b])
        p = float(top_p[b])
        greedy = not (t > 0) or k == 1
        inv_t = 1.0 if greedy else 1.0 / t
        xs = row * inv_t
        M = xs.max()
        logZ = torch.log(torch.exp(xs - M).sum())
        if greedy:
            tok = int(torch.argmax(xs))
            toks[b], lps[b] = tok, float(xs[tok] - M - logZ)
            continue
        keep = torch.ones(V, dtype=torch.bool)
        if 0 < k < V:
            kth = torch.topk(xs, k).values[-1]
            keep &= xs >= kth
        if p < 1.0:
            pm = torch.exp(xs - M) * keep
            order = torch.argsort(xs, descending=True)
            cs = torch.cumsum(pm[order], 0)
            target = p * pm.sum()
            cut = int(torch.searchsorted(cs, target.reshape(1)).item())
            cut = min(cut, V - 1)
            thr = xs[order[cut]]
            keep &= xs >= thr
        u = torch.from_numpy(hash_uniform(int(seeds[b]), np.arange(V, dtype=np.uint64) + np.uint64(int(steps[b]) * V)))
        g = -torch.log(-torch.log(u))
        sc = torch.where(keep, xs + g, torch.tensor(float("-inf")))
        tok = int(torch.argmax(sc))
        toks[b], lps[b] = tok, float(xs[tok] - M - logZ)
    return toks.to(logits.device), lps.to(logits.device)


# ----------------------------------------------------------------------------- search
def score(Q, X, row_bias=None, dot_scale=1.0):
    S = (Q.float() @ X.float().T) * dot_scale
    if row_bias is not None:
        S = S + row_bias.float()[None, :]
    return S


def topk(S: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    k = min(k, S.shape[1])
    v, i = torch.topk(S.float(), k, dim=1)
    return v, i


def ivf_search_topk(Q, X, row_bias, dot_scale, probes, list_beg, list_end, k):
    """Per query: exact top-k over the rows of its probed lists (slab rows; -inf / -1 pads)."""
    nq = Q.shape[0]
    vals = torch.full((nq, k), float("-inf"), device=X.device)
    rows = torch.full((nq, k), -1, dtype=torch.int64, device=X.device)
    beg, end = list_beg.tolist(), list_end.tolist()
    for i in range(nq):
        rr = [torch.arange(beg[p], end[p]) for p in probes[i].tolist() if end[p] > beg[p]]
        if not rr:
            continue
        r = torch.cat(rr).to(X.device)
        s = score(Q[i:i + 1], X.index_select(0, r), None if row_bias is None else row_bias.index_select(0, r),
                  dot_scale)[0]
        kk = min(k, r.numel())
        v, j = torch.topk(s, kk)
        vals[i, :kk] = v
        rows[i, :kk] = r[j]
    return vals, rows


def embedding(ids, table, vocab_lo=0, scale=1.0):
    local = ids.long() - vocab_lo
    ok = (local >= 0) & (local < table.shape[0])
    h = torch.nn.functional.embedding(local.clamp(0, table.shape[0] - 1), table)
    h = h * ok.unsqueeze(-1).to(h.dtype)
    if scale != 1.0:
        h = h * torch.tensor(scale, dtype=h.dtype)
    return h


def pool_l2norm(hidden, cu, mode: int, normalize: bool):
    B = cu.numel() - 1
    out = torch.zeros(B, hidden.shape[1], dtype=torch.float32, device=hidden.device)
    for b in range(B):
        s0, s1 = int(cu[b]), int(cu[b + 1])
        if s1 <= s0:
            continue
        v = hidden[s0].float() if mode == 0 else hidden[s0:s1].float().mean(0)
        if normalize:
            v = v / v.norm().clamp_min(1e-12)
        out[b] = v
    return out


def row_sqnorm(X):
    return X.float().pow(2).sum(-1)


# ---------------------------------------------------------------- DSP (FM-ASR front end)
def fir_c64(x, taps, hist=None):
    """y[i] = sum_k taps[k] x[i-k] (complex x, real taps); x[<0] from ``hist`` or zeros."""
    nt = taps.numel()
    pre = hist if hist is not None else torch.zeros(nt - 1, dtype=x.dtype, device=x.device)
    xx = torch.cat([pre.to(x.dtype), x])
    w = taps.flip(0).to(torch.float64)
    re = torch.nn.functional.conv1d(xx.real.double().view(1, 1, -1), w.view(1, 1, -1)).view(-1)
    im = torch.nn.functional.conv1d(xx.imag.double().view(1, 1, -1), w.view(1, 1, -1)).view(-1)
    return torch.complex(re.float(), im.float())


def fm_demod(x, prev=None):
    if prev is not None:
        x = torch.cat([torch.tensor([prev], dtype=x.dtype, device=x.device), x])
    d = x[1:] * x[:-1].conj()
    return torch.atan2(d.imag, d.real).float()


def resample_pcm(x, h, down, pre, nout, gain):
    """Decimating FIR y[m] = gain * sum_k h[k] x[(m + pre) * down - k]; returns (float, int16)."""
    full = torch.nn.functional.conv1d(
        torch.nn.functional.pad(x.double().view(1, 1, -1), (h.numel() - 1, h.numel() - 1)),
        h.double().flip(0).view(1, 1, -1)).view(-1)
    idx = (torch.arange(nout, dtype=torch.int64) + pre) * down
    y = torch.zeros(nout, dtype=torch.float64)
    ok = idx < full.numel()
    y[ok] = full[idx[ok]]
    y = (gain * y).float()
    pcm = (y * 32768.0).clamp(-32768.0, 32767.0).to(torch.int16)
    return y, pcm


def quant_fp8_rows(x, mode: int, Mp: int):
    """fp32 reference of the row-wise FP8 quantiser (kernels/quant.hip)."""
    xf = x.float()
    if mode == 1:
        F = xf.shape[1] // 2
        g, u = xf[:, :F], xf[:, F:]
        xf = g / (1.0 + torch.exp(-g)) * u
    M, H = xf.shape
    s = xf.abs().amax(1, keepdim=True).clamp_min(1e-12) / 448.0
    y = torch.zeros(Mp, H, dtype=torch.float8_e4m3fn)
    y[:M] = (xf / s).clamp(-448.0, 448.0).to(torch.float8_e4m3fn)
    sp = torch.ones(Mp, 1)
    sp[:M] = s
    return y, sp
