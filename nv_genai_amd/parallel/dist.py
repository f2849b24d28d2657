"""Process-group plumbing: one process per GPU, ``torch.distributed`` with the ``nccl``
backend (RCCL on ROCm) over xGMI; ``gloo`` for CPU-only multi-process tests.

The reference makes no collective calls itself — every collective is implicit inside
TensorRT-LLM/NIM (``tensor_para_size`` / ``enable_custom_all_reduce``,
experimental/fm-asr-streaming-rag/nim/configs/mistral-7b.yaml:32-36) or NeMo.
Here they are explicit: TP all-reduce / all-gather for the decoder, broadcast + all-gather
for the sharded index, and a barrier/max-reduce for benchmark timing.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class ParallelContext:
    world_size: int = 1
    rank: int = 0
    local_rank: int = 0
    tp_size: int = 1
    tp_rank: int = 0
    tp_group: Optional[object] = None
    dp_size: int = 1
    dp_rank: int = 0
    dp_group: Optional[object] = None
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1


_CTX = ParallelContext()


def get_context() -> ParallelContext:
    return _CTX


def env_world() -> tuple:
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0"))))


def init_distributed(tp_size: int = 1, backend: Optional[str] = None,
                     device: Optional[str] = None, timeout_s: int = 600) -> ParallelContext:
    """Initialise the default group from torchrun env vars and build TP/DP subgroups.

    Ranks are laid out TP-major inside a node: ranks [0..tp) form TP group 0, etc., so a TP
    group's all-reduces stay on directly-linked xGMI peers.
    """
    global _CTX
    world, rank, local = env_world()
    use_gpu = torch.cuda.is_available() if device is None else device.startswith("cuda")
    if backend is None:
        backend = "nccl" if use_gpu else "gloo"
    dev = torch.device(f"cuda:{local}") if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(dev)
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kw = {}
        if backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    if world % tp_size != 0:
        raise ValueError(f"world size {world} not divisible by tp {tp_size}")
    dp = world // tp_size
    tp_group = dp_group = None
    if world > 1:
        for d in range(dp):
            ranks = list(range(d * tp_size, (d + 1) * tp_size))
            g = dist.new_group(ranks) if tp_size > 1 else None
            if rank in ranks:
                tp_group = g
        for t in range(tp_size):
            ranks = list(range(t, world, tp_size))
            g = dist.new_group(ranks) if dp > 1 else None
            if rank in ranks:
                dp_group = g
    _CTX = ParallelContext(world_size=world, rank=rank, local_rank=local, tp_size=tp_size,
                           tp_rank=rank % tp_size, tp_group=tp_group, dp_size=dp,
                           dp_rank=rank // tp_size, dp_group=dp_group,
                           backend=backend if world > 1 else "none", device=dev)
    if tp_size > 1 and backend == "nccl" and use_gpu:
        # IPC custom all-reduce for the TP group's small decode messages (RCCL otherwise)
        from .comm import register_custom_all_reduce
        from .custom_ar import maybe_create

        register_custom_all_reduce(tp_group, maybe_create(tp_group, tp_size))
    return _CTX


def set_context(ctx: ParallelContext) -> None:
    global _CTX
    _CTX = ctx


def tp_all_reduce(x: torch.Tensor, ctx: Optional[ParallelContext] = None) -> torch.Tensor:
    ctx = ctx or _CTX
    if ctx.tp_size > 1:
        from .comm import all_reduce

        all_reduce(x, ctx.tp_group)
    return x


def tp_all_gather(x: torch.Tensor, dim: int = -1, ctx: Optional[ParallelContext] = None):
    ctx = ctx or _CTX
    if ctx.tp_size == 1:
        return x
    parts = [torch.empty_like(x) for _ in range(ctx.tp_size)]
    dist.all_gather(parts, x.contiguous(), group=ctx.tp_group)
    return torch.cat(parts, dim=dim)


def barrier():
    if dist.is_initialized():
        if _CTX.backend == "nccl":
            dist.barrier(device_ids=[_CTX.local_rank])
        else:
            dist.barrier()


def all_reduce_max(v: float) -> float:
    if not dist.is_initialized():
        return v
    dev = _CTX.device if _CTX.backend == "nccl" else torch.device("cpu")
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_sum(v: float) -> float:
    if not dist.is_initialized():
        return v
    dev = _CTX.device if _CTX.backend == "nccl" else torch.device("cpu")
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def destroy():
    if dist.is_initialized():
        dist.destroy_process_group()
