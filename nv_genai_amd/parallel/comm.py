"""Collective entry points used by the model code.

``all_reduce`` is RCCL's all-reduce for the TP group. A latency-optimised one-shot
all-reduce for small decode messages over IPC-mapped peer buffers is the planned fast path
for Llama-3-70B TP=8 decode; until it lands every call goes to RCCL, whose
ring/tree selection over the 7 xGMI links is used as-is.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def all_reduce(x: torch.Tensor, group=None) -> torch.Tensor:
    dist.all_reduce(x, op=dist.ReduceOp.SUM, group=group)
    return x


def broadcast(x: torch.Tensor, src: int, group=None) -> torch.Tensor:
    dist.broadcast(x, src=src, group=group)
    return x


def all_gather_cat(x: torch.Tensor, world: int, dim: int = 0, group=None) -> torch.Tensor:
    parts = [torch.empty_like(x) for _ in range(world)]
    dist.all_gather(parts, x.contiguous(), group=group)
    return torch.cat(parts, dim=dim)
