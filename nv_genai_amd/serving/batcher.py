"""Dynamic batcher for the embedding / reranking engines: concurrent requests arriving within
``max_delay_s`` are merged into one packed encoder forward (Triton dynamic batching with
``max_queue_delay``, experimental/streaming_ingest_rag/docker/extras/all-MiniLM-L6-v2_config.pbtxt:25-36,
with preferred sizes replaced by a token budget since sequences are packed, not padded).
"""
from __future__ import annotations

import queue
import threading
import time
from concurrent.futures import Future
from typing import List, Sequence, Tuple

import torch


class DynamicBatcher:
    """Results are host fp32 tensors. On a GPU the encoder runs on the batcher's own HIP stream
    and its output comes back through pinned memory, waited for on the batcher thread: a model
    server that also runs an LLM engine would otherwise queue every embedding behind the LLM
    step in flight on the default stream, and a ``.cpu()`` on the event loop would block the
    loop (every open stream) until that step ends (profiles/r5_http/: 12 s of 80 in the
    split topology)."""

    def __init__(self, engine, max_delay_s: float = 0.002, max_batch_texts: int = 1024):
        self.engine = engine
        self.max_delay_s = max_delay_s
        self.max_batch_texts = max_batch_texts
        self.q: "queue.Queue[Tuple[List[List[int]], Future]]" = queue.Queue()
        self.batches = 0
        dev = getattr(engine, "device", None)
        self.stream = torch.cuda.Stream(dev) if isinstance(dev, torch.device) and dev.type == "cuda" else None
        self.thread = threading.Thread(target=self._run, daemon=True, name="embed-batcher")
        self.thread.start()

    def _embed_host(self, seqs: List[List[int]]) -> torch.Tensor:
        if self.stream is None:
            return self.engine.embed_ids(seqs).cpu()
        with torch.cuda.stream(self.stream):
            out = self.engine.embed_ids(seqs)
            host = torch.empty(out.shape, dtype=out.dtype, pin_memory=True)
            host.copy_(out, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        ev.synchronize()
        return host

    def submit_ids(self, seqs: List[List[int]]) -> Future:
        f: Future = Future()
        self.q.put((seqs, f))
        return f

    def embed(self, texts: Sequence[str], input_type: str = "passage", truncate: str = "END") -> torch.Tensor:
        return self.submit_ids(self.engine.tokenize(texts, input_type, truncate)).result()

    def _run(self):
        while True:
            items = [self.q.get()]
            n = len(items[0][0])
            deadline = time.monotonic() + self.max_delay_s
            while n < self.max_batch_texts:
                rem = deadline - time.monotonic()
                if rem <= 0:
                    break
                try:
                    it = self.q.get(timeout=rem)
                except queue.Empty:
                    break
                items.append(it)
                n += len(it[0])
            seqs = [s for it, _ in items for s in it]
            try:
                out = self._embed_host(seqs)
                self.batches += 1
                i = 0
                for it, fut in items:
                    fut.set_result(out[i:i + len(it)])
                    i += len(it)
            except Exception as e:  # noqa: BLE001
                for _, fut in items:
                    if not fut.done():
                        fut.set_exception(e)
