"""Per-shape GEMM solution selection for the library GEMMs (hipBLASLt / rocBLAS).

The projections of the LLM and encoder are plain ``x @ W^T`` GEMMs, which stay on the vendor
libraries. Their default heuristic is poor for two regimes that dominate serving:

* decode (M = padded batch 1..256, N up to 28672, K 4096/14336): too few tiles and no
  split-K at N = 4096 leave most of the 256 CUs idle;
* prefill chunks (M = 16384): the heuristic's MT256x256 macro-tile reaches ≈1.7 PFLOP/s, the
  best solution ≈2.1 PFLOP/s on gfx950.

``scripts/tune_gemms.py`` benchmarks every hipBLASLt/rocBLAS solution for the exact shapes
the engine issues (the decode graph buckets and the prefill chunk size) on an MI355X and
writes a PyTorch TunableOp results file under ``assets/tunableop/``. ``use_tuned_gemms``
loads it with tuning off, so serving never tunes online; shapes not in the file keep the
library default.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

ASSET_DIR = os.path.join(os.path.dirname(os.path.dirname(__file__)), "assets", "tunableop")
DEFAULT_FILE = os.path.join(ASSET_DIR, "gemm_gfx950.csv")
_loaded: Optional[str] = None


def use_tuned_gemms(path: Optional[str] = None) -> bool:
    """Enable TunableOp lookups from ``path`` (default: the shipped gfx950 table). Returns
    whether a table was loaded. No-op on CPU or when the table is missing."""
    global _loaded
    if not torch.cuda.is_available() or torch.version.hip is None:
        return False
    path = path or os.environ.get("NGA_GEMM_TABLE", DEFAULT_FILE)
    if _loaded == path:
        return True
    if not os.path.exists(path):
        return False
    import torch.cuda.tunable as tn

    tn.enable(True)
    tn.tuning_enable(False)
    tn.record_untuned_enable(False)
    ok = tn.read_file(path)
    if not ok:
        tn.enable(False)
        return False
    _loaded = path
    return True


def llm_gemm_shapes(cfg, tp: int = 1, decode_sizes=(), prefill_tokens=()):
    """(M, N, K) of every projection GEMM the LLM issues for the given M values."""
    H, I, D = cfg.hidden, cfg.ffn, cfg.head_dim
    mats = [(cfg.qkv_dim // tp, H), (H, cfg.heads * D // tp), (2 * I // tp, H), (H, I // tp)]
    out = []
    for m in list(decode_sizes) + list(prefill_tokens):
        out += [(m, n, k) for n, k in mats]
    for m in decode_sizes:
        out.append((m, cfg.vocab_size // tp, H))
    return out


def encoder_gemm_shapes(cfg, tokens=()):
    H, I = cfg.hidden, cfg.ffn
    mats = [(3 * H, H), (H, H), (I, H), (H, I)]
    return [(m, n, k) for m in tokens for n, k in mats]
