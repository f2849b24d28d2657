"""Collective entry points used by the model code.

``all_reduce`` takes the group's custom all-reduce (:mod:`.custom_ar`: one-shot / two-shot
direct reads of IPC-mapped peer buffers over all 7 xGMI links) when one is
registered and the tensor fits it, and RCCL otherwise (CPU/gloo tensors, oversized or
misaligned messages, or a group whose custom all-reduce failed its self-test).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


_CUSTOM = {}


def register_custom_all_reduce(group, car) -> None:
    """Route ``all_reduce`` calls on ``group`` through ``car`` when it can take them."""
    if car is None:
        _CUSTOM.pop(id(group), None)
    else:
        _CUSTOM[id(group)] = car


def custom_all_reduce_for(group):
    return _CUSTOM.get(id(group))


def all_reduce(x: torch.Tensor, group=None) -> torch.Tensor:
    car = _CUSTOM.get(id(group))
    if car is not None and car.eligible(x):
        return car.all_reduce(x)
    dist.all_reduce(x, op=dist.ReduceOp.SUM, group=group)
    return x


def broadcast(x: torch.Tensor, src: int, group=None) -> torch.Tensor:
    dist.broadcast(x, src=src, group=group)
    return x


def all_gather_cat(x: torch.Tensor, world: int, dim: int = 0, group=None) -> torch.Tensor:
    parts = [torch.empty_like(x) for _ in range(world)]
    dist.all_gather(parts, x.contiguous(), group=group)
    return torch.cat(parts, dim=dim)
