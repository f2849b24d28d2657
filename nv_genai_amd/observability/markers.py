"""ROCTx ranges around the engine's GPU phases (SURVEY.md §5.1 "roctx ranges around
prefill/decode/embed/search steps"). On ROCm ``torch.cuda.nvtx`` emits roctx markers, which
``rocprofv3 --marker-trace`` records next to the kernel trace, so a timeline shows which
scheduler step (prefill / mixed / decode), embedding batch or index search each kernel
belongs to. Off by default (one Python call per range); ``NGA_MARKERS=1`` turns them on.
"""
from __future__ import annotations

import contextlib
import os

import torch

ENABLED = os.environ.get("NGA_MARKERS", "0") == "1" and torch.cuda.is_available()


@contextlib.contextmanager
def gpu_range(name: str):
    if not ENABLED:
        yield
        return
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()
