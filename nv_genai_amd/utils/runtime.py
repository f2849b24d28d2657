"""Host-runtime tuning for the serving loop.

CPython's cyclic garbage collector walks every tracked object in a generation when it runs.
A serving process holds hundreds of thousands of long-lived objects (requests, token lists,
detokenizer tables, docstore caches); a full collection of them is a multi-millisecond
stop-the-world pause on the thread that launches GPU steps, and the GPU idles for exactly
that long (rocprofv3 gap analysis of the closed-loop bench: idle gaps of 3.5-8 ms between
the copies that start an engine step — scripts/gap_analysis.py).

``quiet_gc`` moves everything alive after start-up into the permanent generation
(``gc.freeze``) so collections only scan objects created while serving, and raises the
generation-0 threshold so short-lived per-step garbage is collected in fewer, equally small
passes. Reference counting still frees acyclic garbage immediately.
"""
from __future__ import annotations

import contextlib
import gc
import threading

# Held while a thread captures a hipGraph, and by the other components of a serving process
# that issue library GEMMs from their own threads (the embedding / reranking encoder). The first
# use of a hipBLASLt solution in a thread runs set-up operations that are not permitted while
# another thread's stream is capturing (hipErrorStreamCaptureImplicit / ...Unsupported from
# hipblaslt.cpp, which invalidates the capture: scripts/dev/capture_race.py). Captures are rare
# (one per new graph bucket), so the lock is almost always free.
GPU_CAPTURE_LOCK = threading.RLock()


@contextlib.contextmanager
def capture_guard():
    with GPU_CAPTURE_LOCK:
        yield


def quiet_gc(gen0_threshold: int = 50_000) -> None:
    gc.collect()
    gc.freeze()
    _, g1, g2 = gc.get_threshold()
    gc.set_threshold(gen0_threshold, max(g1, 20), max(g2, 100))
