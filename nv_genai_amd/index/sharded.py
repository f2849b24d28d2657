"""Vector index sharded across ranks (kernel K15): the 10M-vector
index of the query-decomposition config split over the 8 GPUs of a node.

* ``add``: every rank sees the same (vectors, ids) and keeps its stripe (row i -> rank
  i % world), so no data moves at build time;
* ``search``: the driver's query block is broadcast (RCCL broadcast, CC7), each rank runs the
  MFMA score + top-k kernels on its local shard, the per-shard (score, id) lists are
  all-gathered (CC8) and merged by the same top-k kernel over the world*k candidates (K15).
At 1.25M x 1024 bf16 per GPU a shard is 2.5 GB of HBM; each collective moves a few KB.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist

from .. import ops
from ..parallel.dist import ParallelContext, get_context
from .flat import FlatIndex


class ShardedIndex:
    def __init__(self, dim: int, metric: str = "cosine", device: Optional[str] = None,
                 pctx: Optional[ParallelContext] = None, group=None, capacity: int = 1024):
        self.p = pctx or get_context()
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.dim, self.metric = dim, metric
        self.local = FlatIndex(dim, metric, device, capacity=capacity)
        self.comm_dev = self.local.device if self.p.backend == "nccl" else torch.device("cpu")

    def __len__(self):
        n = torch.tensor([len(self.local)], dtype=torch.int64, device=self.comm_dev)
        if self.world > 1:
            dist.all_reduce(n, group=self.group)
        return int(n.item())

    def add(self, vecs: torch.Tensor, ids: torch.Tensor) -> None:
        sel = torch.arange(vecs.shape[0]) % self.world == self.rank
        self.local.add(vecs[sel], ids[sel])

    def add_random(self, n_total: int, seed: int = 0) -> None:
        """Each rank generates only its own stripe of a synthetic index; global ids are
        striped like ``add`` (row i of rank r is id ``i * world + r``)."""
        n_local = n_total // self.world + (1 if self.rank < n_total % self.world else 0)
        self.local.add_random(n_local, seed=seed * 1009 + self.rank, first_id=self.rank, id_stride=self.world)

    def remove(self, ids) -> int:
        return self.local.remove(ids)

    @torch.inference_mode()
    def search(self, q: torch.Tensor, k: int, src: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
        if q.dim() == 1:
            q = q.unsqueeze(0)
        if self.world == 1:
            return self.local.search(q, k)
        qd = q.to(self.comm_dev, torch.float32).contiguous()
        dist.broadcast(qd, src=src, group=self.group)
        vals, ids = self.local.search(qd.to(self.local.device), k)
        nq = qd.shape[0]
        kk = vals.shape[1]
        if kk < k:  # pad a short shard
            vals = torch.cat([vals, torch.full((nq, k - kk), float("-inf"), device=vals.device)], 1)
            ids = torch.cat([ids, torch.full((nq, k - kk), -1, dtype=torch.int64, device=ids.device)], 1)
        v_all = [torch.empty(nq, k, dtype=torch.float32, device=self.comm_dev) for _ in range(self.world)]
        i_all = [torch.empty(nq, k, dtype=torch.int64, device=self.comm_dev) for _ in range(self.world)]
        dist.all_gather(v_all, vals.to(self.comm_dev).float().contiguous(), group=self.group)
        dist.all_gather(i_all, ids.to(self.comm_dev).contiguous(), group=self.group)
        cv = torch.cat(v_all, 1).to(self.local.device).contiguous()
        ci = torch.cat(i_all, 1).to(self.local.device).contiguous()
        if cv.is_cuda:
            mv = torch.empty(nq, k, dtype=torch.float32, device=cv.device)
            mi = torch.empty(nq, k, dtype=torch.int64, device=cv.device)
            ops.kernels().topk(cv, ci, cv.shape[1], k, mv, mi)
            return mv, mi
        mv, pos = torch.topk(cv, k, dim=1)
        return mv, torch.gather(ci, 1, pos)
