"""Selection of the decode-shape projection GEMM (csrc/kernels/gemm_skinny.hip) per call.

``assets/skinny_gemm_gfx950.json`` (written by ``benchmarks/skinny_table.py`` on an MI355X) maps
each projection shape ``"{N}x{K}"`` and row count M to the measured winner: ``[cfg, split]`` of
the skinny kernel or ``"lib"`` (the library GEMM). Each entry was timed together with the kernel
that consumes its output in the model (the residual add + RMSNorm for o / down, SwiGLU for
gate / up, fp32 logits for the LM head), so a choice is an end-to-end one. A call with M between
table rows takes the next larger row (the engine's graph buckets are table rows); shapes not in
the table, and M above its largest row, use the library GEMM.

``NGA_SKINNY=0`` turns the path off (A/B runs); ``NGA_SKINNY_TABLE`` points at another table.
"""
from __future__ import annotations

import bisect
import json
import os
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import torch

ASSET = os.path.join(os.path.dirname(os.path.dirname(__file__)), "assets", "skinny_gemm_gfx950.json")


@dataclass
class PartialSum:
    """K-split fp32 partial products [S, M, N] of a projection; the consumer sums the slabs
    (``ops.splitk_add_rmsnorm`` folds the sum into the residual add + RMSNorm)."""

    slabs: torch.Tensor

    @property
    def shape(self):
        return self.slabs.shape[1:]

    def materialize(self) -> torch.Tensor:
        from . import splitk_reduce

        return splitk_reduce(self.slabs)


class SkinnyTable:
    def __init__(self, path: Optional[str] = None):
        self.path = path or os.environ.get("NGA_SKINNY_TABLE", ASSET)
        self.shapes: Dict[Tuple[int, int], Tuple[list, list]] = {}
        if os.path.exists(self.path):
            with open(self.path) as f:
                doc = json.load(f)
            for key, ent in doc.get("table", {}).items():
                n, k = (int(v) for v in key.split("x"))
                ms = sorted(int(m) for m in ent["by_m"])
                self.shapes[(n, k)] = (ms, [ent["by_m"][str(m)] for m in ms])

    def pick(self, N: int, K: int, M: int) -> Optional[Tuple[int, int]]:
        """(cfg, split) for out[M, N] = x[M, K] @ W^T, or None for the library GEMM."""
        ent = self.shapes.get((N, K))
        if ent is None or M < 1:
            return None
        ms, choice = ent
        i = bisect.bisect_left(ms, M)
        if i == len(ms):
            return None
        c = choice[i]
        return None if c == "lib" else (int(c[0]), int(c[1]))


_TABLE: Optional[SkinnyTable] = None


def table() -> SkinnyTable:
    global _TABLE
    if _TABLE is None:
        _TABLE = SkinnyTable()
    return _TABLE


def enabled() -> bool:
    return os.environ.get("NGA_SKINNY", "1") != "0"
