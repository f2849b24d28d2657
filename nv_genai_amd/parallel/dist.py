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
    pp_size: int = 1
    pp_rank: int = 0
    mp_group: Optional[object] = None   # every rank of one model replica (tp x pp)
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1

    @property
    def mp_size(self) -> int:
        return self.tp_size * self.pp_size

    @property
    def mp_src(self) -> int:
        """Global rank of the replica's driver (pp stage 0, tp rank 0)."""
        return self.rank - self.pp_rank * self.tp_size - self.tp_rank

    @property
    def pp_prev(self) -> int:
        return self.rank - self.tp_size

    @property
    def pp_next(self) -> int:
        return self.rank + self.tp_size

    @property
    def pp_first_rank(self) -> int:
        """Global rank of this tp rank's peer on pipeline stage 0."""
        return self.rank - self.pp_rank * self.tp_size

    @property
    def pp_last_rank(self) -> int:
        return self.pp_first_rank + (self.pp_size - 1) * self.tp_size


_CTX = ParallelContext()
PLACEMENT = None   # utils.affinity.Placement of this rank (multi-rank GPU jobs)


def bind_numa(world: Optional[int] = None) -> None:
    """Bind this rank's threads to its GPU's NUMA node (utils/affinity.py). Must run before the
    first HIP call of the process — it only counts devices through sysfs — so threads the HIP
    runtime starts inherit the mask. Once per process; single-rank jobs are left alone."""
    global PLACEMENT
    if PLACEMENT is not None:
        return
    w, _, local = env_world() if world is None else (world, 0, int(os.environ.get("LOCAL_RANK", "0")))
    if w <= 1:
        return
    from ..utils.affinity import bind_local_rank

    PLACEMENT = bind_local_rank(local, int(os.environ.get("LOCAL_WORLD_SIZE", w)))


def get_context() -> ParallelContext:
    return _CTX


def env_world() -> tuple:
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0"))))


def init_distributed(tp_size: int = 1, backend: Optional[str] = None,
                     device: Optional[str] = None, timeout_s: int = 600,
                     pp_size: int = 1) -> ParallelContext:
    """Initialise the default group from torchrun env vars and build TP/PP/DP subgroups.

    Ranks are laid out TP-major, then pipeline stage, then replica:
    ``rank = dp_rank * (tp * pp) + pp_rank * tp + tp_rank``. A TP group's all-reduces stay
    on directly-linked xGMI peers; pipeline stage s sends activations to the same tp rank of
    stage s + 1 (``rank + tp``); a replica's tp x pp ranks form its model-parallel group.
    """
    global _CTX
    world, rank, local = env_world()
    if world > 1 and (device is None or device.startswith("cuda")):
        bind_numa()   # before torch.cuda.is_available() starts the HIP runtime's threads
    use_gpu = torch.cuda.is_available() if device is None else device.startswith("cuda")
    ngpu = torch.cuda.device_count() if use_gpu else 0
    # ranks on THIS node against its GPUs (a multi-node job has world > device_count on
    # every node and must stay on RCCL)
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    oversubscribed = use_gpu and local_world > ngpu
    if oversubscribed:
        # more local ranks than GPUs (a multi-rank rehearsal on a 1-GPU box): ranks share
        # devices round-robin and the host-side groups go over gloo, since RCCL refuses two
        # ranks of one communicator on the same device. An 8-GPU node never takes this path.
        local = local % max(1, ngpu)
        if backend is None:
            backend = "gloo"
        if rank == 0:
            print(f"[nga] {world} ranks on {ngpu} GPU(s): ranks share devices, {backend} backend",
                  flush=True)
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
        # one key namespace per elastic incarnation: after a group restart (torchrun
        # --max-restarts) the rendezvous store still holds the dead ranks' gloo/RCCL
        # addresses, and a fresh rank must not connect to those
        td = datetime.timedelta(seconds=timeout_s)
        store, _, _ = next(dist.rendezvous("env://", rank, world, timeout=td))
        store = dist.PrefixStore(f"nga{os.environ.get('TORCHELASTIC_RESTART_COUNT', '0')}/", store)
        dist.init_process_group(backend=backend, store=store, rank=rank, world_size=world,
                                timeout=td, **kw)
    mp = tp_size * pp_size
    if world % mp != 0:
        raise ValueError(f"world size {world} not divisible by tp {tp_size} x pp {pp_size}")
    dp = world // mp
    tp_group = dp_group = mp_group = None
    if world > 1:
        # new_group is collective over the default group: every rank creates every group
        for d in range(dp):
            for s_ in range(pp_size):
                ranks = [d * mp + s_ * tp_size + t for t in range(tp_size)]
                g = dist.new_group(ranks) if tp_size > 1 else None
                if rank in ranks:
                    tp_group = g
        for d in range(dp):
            ranks = list(range(d * mp, (d + 1) * mp))
            g = dist.new_group(ranks) if mp > 1 else None
            if rank in ranks:
                mp_group = g
        for j in range(mp):
            ranks = list(range(j, world, mp))
            g = dist.new_group(ranks) if dp > 1 else None
            if rank in ranks:
                dp_group = g
    _CTX = ParallelContext(world_size=world, rank=rank, local_rank=local, tp_size=tp_size,
                           tp_rank=rank % tp_size, tp_group=tp_group, dp_size=dp,
                           dp_rank=rank // mp, dp_group=dp_group, pp_size=pp_size,
                           pp_rank=(rank % mp) // tp_size, mp_group=mp_group,
                           backend=backend if world > 1 else "none", device=dev)
    if tp_size > 1 and use_gpu:
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
    if x.is_cuda and x.dim() == 2 and dim in (-1, 1):
        # the IPC all-gather (direct peer reads over xGMI; capture-safe with any backend)
        from .comm import custom_all_reduce_for

        car = custom_all_reduce_for(ctx.tp_group)
        if car is not None and car.gather_eligible(x):
            return car.all_gather(x)
    y = x.contiguous()
    if ctx.backend == "gloo" and y.is_cuda:   # gloo gathers host tensors
        y = y.cpu()
    parts = [torch.empty_like(y) for _ in range(ctx.tp_size)]
    dist.all_gather(parts, y, group=ctx.tp_group)
    return torch.cat(parts, dim=dim).to(x.device)


def tp_reduce_scatter_rows(x: torch.Tensor, ctx: Optional[ParallelContext] = None) -> torch.Tensor:
    """Sum of ``x`` [T, H] over the TP group, keeping only this rank's T / tp rows
    (sequence parallelism: replaces the all-reduce after a row-parallel GEMM)."""
    ctx = ctx or _CTX
    tp = ctx.tp_size
    if tp == 1:
        return x
    rows = x.shape[0] // tp
    if ctx.backend == "nccl":
        out = torch.empty(rows, *x.shape[1:], dtype=x.dtype, device=x.device)
        dist.reduce_scatter_tensor(out, x.contiguous(), group=ctx.tp_group)
        return out
    # gloo has no reduce-scatter: all-reduce on the host, keep our slice
    y = x.contiguous().cpu() if x.is_cuda else x.contiguous().clone()
    dist.all_reduce(y, group=ctx.tp_group)
    return y[ctx.tp_rank * rows:(ctx.tp_rank + 1) * rows].to(x.device)


def tp_all_gather_rows(x: torch.Tensor, ctx: Optional[ParallelContext] = None) -> torch.Tensor:
    """Concatenate every TP rank's row shard [T / tp, H] into [T, H] (rank order)."""
    ctx = ctx or _CTX
    tp = ctx.tp_size
    if tp == 1:
        return x
    if ctx.backend == "nccl":
        out = torch.empty(x.shape[0] * tp, *x.shape[1:], dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(out, x.contiguous(), group=ctx.tp_group)
        return out
    return tp_all_gather(x, dim=0, ctx=ctx)


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


def all_gather_objects(obj) -> list:
    """Every rank's ``obj`` in rank order (``[obj]`` outside a job)."""
    if not dist.is_initialized():
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def destroy():
    if dist.is_initialized():
        dist.destroy_process_group()
