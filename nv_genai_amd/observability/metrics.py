"""Prometheus-text metrics (QPS, TTFT, TPOT, queue depth, batch size, KV
utilisation, index latency, HBM use). A lock-protected registry of counters and
summaries (count / sum / p50 / p95 over a sliding window) rendered in exposition format.
"""
from __future__ import annotations

import threading
from collections import deque
from typing import Dict, Optional


class Registry:
    def __init__(self, window: int = 4096):
        self.lock = threading.Lock()
        self.counters: Dict[str, float] = {}
        self.samples: Dict[str, deque] = {}
        self.sums: Dict[str, float] = {}
        self.counts: Dict[str, int] = {}
        self.window = window

    def inc(self, name: str, v: float = 1.0):
        with self.lock:
            self.counters[name] = self.counters.get(name, 0.0) + v

    def observe(self, name: str, v: float):
        with self.lock:
            d = self.samples.get(name)
            if d is None:
                d = self.samples[name] = deque(maxlen=self.window)
            d.append(v)
            self.sums[name] = self.sums.get(name, 0.0) + v
            self.counts[name] = self.counts.get(name, 0) + 1

    def quantile(self, name: str, q: float) -> Optional[float]:
        with self.lock:
            d = sorted(self.samples.get(name, ()))
        if not d:
            return None
        return d[min(len(d) - 1, int(q * len(d)))]

    def render(self, gauges: Optional[dict] = None, prefix: str = "nga") -> str:
        out = []
        with self.lock:
            for k, v in sorted(self.counters.items()):
                out.append(f"# TYPE {prefix}_{k} counter\n{prefix}_{k} {v}")
            names = sorted(self.samples)
        for k in names:
            out.append(f"# TYPE {prefix}_{k} summary")
            for q in (0.5, 0.95, 0.99):
                v = self.quantile(k, q)
                out.append(f'{prefix}_{k}{{quantile="{q}"}} {v if v is not None else "NaN"}')
            out.append(f"{prefix}_{k}_sum {self.sums.get(k, 0.0)}")
            out.append(f"{prefix}_{k}_count {self.counts.get(k, 0)}")
        for k, v in sorted((gauges or {}).items()):
            if isinstance(v, (int, float)):
                out.append(f"# TYPE {prefix}_{k} gauge\n{prefix}_{k} {v}")
        for k, v in sorted(hbm_gauges().items()):
            out.append(f"# TYPE {prefix}_{k} gauge\n{prefix}_{k} {v}")
        return "\n".join(out) + "\n"


def hbm_gauges() -> dict:
    try:
        import torch

        if not torch.cuda.is_available():
            return {}
        free, total = torch.cuda.mem_get_info()
        return {"hbm_used_bytes": total - free, "hbm_total_bytes": total,
                "torch_allocated_bytes": torch.cuda.memory_allocated()}
    except Exception:  # noqa: BLE001
        return {}


METRICS = Registry()
