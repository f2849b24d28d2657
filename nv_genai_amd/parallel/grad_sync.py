"""Bucketed data-parallel gradient all-reduce, overlapped with backward.

Parameters are grouped, in reverse registration order (≈ the order backward produces their
gradients), into flat fp32 buckets of ``bucket_mb``. A post-accumulate-grad hook counts the
gradients that have landed in each bucket; when a bucket is complete its gradients are
copied into the flat buffer and an async all-reduce is launched right away, so RCCL moves
bucket i over xGMI while backward is still computing bucket i+1. ``finish()`` waits for the
outstanding collectives and scatters the averaged buckets back into ``.grad``.

xGMI rings are per-link bound (≈153 GB/s per link), so a few large buckets beat many small
ones: the default 256 MB bucket is ≈2 ms of ring time at 8 GPUs, long enough to hide the
launch latency, short enough to overlap with the backward of a transformer block.

With gradient accumulation call ``sync(False)`` for the micro-steps that should not
communicate (like DDP's ``no_sync``).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch
import torch.distributed as dist


class GradBucketer:
    def __init__(self, params: Sequence[torch.Tensor], group=None, bucket_mb: float = 256.0):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.enabled = True
        cap = int(bucket_mb * 2 ** 20) // 4
        self.buckets: List[List[torch.Tensor]] = []
        cur, size = [], 0
        for p in reversed(self.params):
            if cur and size + p.numel() > cap:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += p.numel()
        if cur:
            self.buckets.append(cur)
        self.index = {}
        for bi, b in enumerate(self.buckets):
            for p in b:
                self.index[id(p)] = bi
        self.flat = [torch.zeros(sum(p.numel() for p in b), dtype=torch.float32, device=b[0].device)
                     for b in self.buckets]
        self._reset()
        self._hooks = [p.register_post_accumulate_grad_hook(self._hook) for p in self.params] \
            if self.world > 1 else []

    def _reset(self):
        self.ready = [0] * len(self.buckets)
        self.works: List[Optional[object]] = [None] * len(self.buckets)

    def sync(self, enabled: bool) -> None:
        self.enabled = enabled

    def _hook(self, p: torch.Tensor) -> None:
        if not self.enabled:
            return
        bi = self.index[id(p)]
        self.ready[bi] += 1
        if self.ready[bi] == len(self.buckets[bi]):
            self._launch(bi)

    def _launch(self, bi: int) -> None:
        flat, o = self.flat[bi], 0
        for p in self.buckets[bi]:
            n = p.numel()
            if p.grad is None:
                flat[o:o + n].zero_()
            else:
                flat[o:o + n].copy_(p.grad.reshape(-1))
            o += n
        self.works[bi] = dist.all_reduce(flat, group=self.group, async_op=True)

    def finish(self) -> None:
        """Wait for every bucket (launching any whose hooks did not all fire, e.g. unused
        parameters) and write the averaged gradients back."""
        if self.world == 1:
            return
        for bi in range(len(self.buckets)):
            if self.works[bi] is None:
                self._launch(bi)
        for bi, w in enumerate(self.works):
            w.wait()
            flat, o = self.flat[bi], 0
            flat.div_(self.world)
            for p in self.buckets[bi]:
                n = p.numel()
                g = flat[o:o + n].view_as(p).to(p.dtype)
                if p.grad is None:
                    p.grad = g.clone()
                else:
                    p.grad.copy_(g)
                o += n
        self._reset()

    def remove(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []


def broadcast_params(params: Sequence[torch.Tensor], src: int = 0, group=None) -> None:
    """Make every rank start from rank ``src``'s parameters."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    with torch.no_grad():
        for p in params:
            dist.broadcast(p.data, src=src, group=group)
