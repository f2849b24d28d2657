"""Vector index sharded across ranks (kernel K15): the 10M-vector
index of the query-decomposition config split over the 8 GPUs of a node.

* ``add``: every rank sees the same (vectors, ids) and keeps its stripe (row i -> rank
  i % world), so no data moves at build time;
* ``search``: the driver's query block reaches every rank (inside the replica's step-channel
  command, or by a broadcast, CC7), each rank runs the MFMA score + top-k kernels on its local
  shard, the per-shard (score, id) lists are packed into one tensor and all-gathered in one
  collective — the IPC all-gather kernel of the TP group when it has one (CC8) — and merged by
  the same top-k kernel over the world*k candidates (K15).
At 1.25M x 1024 bf16 per GPU a shard is 2.5 GB of HBM; the gather moves 48 B per query and rank.

Snapshot / restore (the Milvus-volume / FAISS ``save_local`` persistence of
the reference, ``docker-compose-vectordb.yaml:27,46,64``): ``save`` writes one safetensors
shard per rank into a fresh generation directory and rank 0 then publishes ``manifest.json``
with an atomic rename, so a crash mid-save leaves the previous snapshot intact. ``load``
restores the shard of each rank directly when the world size matches, and re-stripes the rows
(global row g -> rank g % world, same rule as ``add``) when it does not.
"""
from __future__ import annotations

import json
import os
import shutil
import time
from pathlib import Path
from typing import Optional, Tuple

import numpy as np  # noqa: F401  (query_payload's return type)

import torch
import torch.distributed as dist

from .. import ops
from ..parallel.dist import ParallelContext, get_context
from .flat import FlatIndex


class ShardedIndex:
    def __init__(self, dim: int, metric: str = "cosine", device: Optional[str] = None,
                 pctx: Optional[ParallelContext] = None, group=None, capacity: int = 1024,
                 ipc_gather: bool = True):
        self.p = pctx or get_context()
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.dim, self.metric = dim, metric
        self.local = FlatIndex(dim, metric, device, capacity=capacity)
        self.comm_dev = self.local.device if self.p.backend == "nccl" else torch.device("cpu")
        # searches, how their results were gathered, host time inside search() (launch-side:
        # the merge is left on the stream)
        self.stats = {"searches": 0, "broadcasts": 0, "ipc_gathers": 0, "pg_gathers": 0, "host_s": 0.0}
        self._car = self._make_ipc_gather() if ipc_gather else None
        # searches whose query block comes from the host (the step-channel command) run on
        # their own stream: they start beside the replica's in-flight step instead of queueing
        # behind it, and the engine's stream never waits for them (search_side)
        self._stream = torch.cuda.Stream(self.local.device) if self.local.device.type == "cuda" else None

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

    # ------------------------------------------------------------------ persistence
    def _obj_broadcast(self, obj):
        if self.world == 1:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=0, group=self.group)
        return box[0]

    def _obj_gather(self, obj):
        if self.world == 1:
            return [obj]
        out = [None] * self.world
        dist.all_gather_object(out, obj, group=self.group)
        return out

    def _barrier(self):
        if self.world > 1:
            dist.barrier(group=self.group)

    def save(self, path: str, keep: int = 1) -> dict:
        """Collective: every rank of the group calls it with the same (shared-filesystem) path.
        Returns the manifest. ``keep`` older generations are retained besides the new one."""
        root = Path(path)
        gen = self._obj_broadcast(f"gen-{time.time_ns():020d}")
        self.local.save(str(root / gen / f"shard-{self.rank:04d}"))
        n = len(self.local)
        counts = self._obj_gather(n)
        manifest = {"kind": "sharded", "generation": gen, "world": self.world, "dim": self.dim,
                    "metric": self.metric, "counts": counts, "total": int(sum(counts)),
                    "shards": [f"{gen}/shard-{r:04d}" for r in range(self.world)]}
        self._barrier()  # every shard is on disk before the manifest points at it
        if self.rank == 0:
            tmp = root / "manifest.json.tmp"
            tmp.write_text(json.dumps(manifest, indent=1))
            os.replace(tmp, root / "manifest.json")
            gens = sorted(d.name for d in root.iterdir() if d.is_dir() and d.name.startswith("gen-"))
            for old in [g for g in gens if g != gen][: max(0, len(gens) - 1 - keep)]:
                shutil.rmtree(root / old, ignore_errors=True)
        self._barrier()
        return manifest

    @classmethod
    def load(cls, path: str, device: Optional[str] = None, pctx: Optional[ParallelContext] = None,
             group=None) -> "ShardedIndex":
        """Collective. Restores the snapshot ``manifest.json`` points at, re-striping the rows
        when the group size differs from the one that saved it."""
        root = Path(path)
        manifest = json.loads((root / "manifest.json").read_text())
        if manifest.get("kind") != "sharded":
            raise ValueError(f"{root}: not a sharded-index snapshot")
        idx = cls(manifest["dim"], manifest["metric"], device, pctx=pctx, group=group)
        if manifest["world"] == idx.world:
            idx.local = FlatIndex.load(str(root / manifest["shards"][idx.rank]), device)
            got = len(idx.local)
            if got != manifest["counts"][idx.rank]:
                raise ValueError(f"shard {idx.rank}: {got} rows, manifest says "
                                 f"{manifest['counts'][idx.rank]}")
            return idx
        # re-stripe: the saved global order is shard-major with saved row j of shard s at
        # global row j * world_saved + s; keep rows whose global row maps to this rank
        ws = manifest["world"]
        for s, rel in enumerate(manifest["shards"]):
            shard = FlatIndex.load(str(root / rel), "cpu")
            n = shard.n
            live = shard.bias[:n] != float("-inf")
            g = torch.arange(n) * ws + s
            sel = live & (g % idx.world == idx.rank)
            if bool(sel.any()):  # stored rows are already prepared; add() re-derives the bias
                idx.local.add(shard.X[:n][sel], shard.ids[:n][sel])
        return idx

    def _make_ipc_gather(self):
        """This index's own IPC communicator (parallel/custom_ar.py: Signal block + staging
        buffers mapped by every rank of the group), used only for the search gather. Its own,
        not the TP group's: a search may run on another stream than the model's all-reduces
        (bench.py's retrieval stream), and two kernels of one communicator must never run at
        once on a rank (they share its call counter). Collective over the group; None on the
        CPU, at world 1, with NGA_CUSTOM_AR=0, or when it fails its self-test."""
        if (self.world <= 1 or self.world > 8 or self.local.device.type != "cuda"
                or os.environ.get("NGA_CUSTOM_AR", "1") == "0"):
            return None
        from ..parallel.custom_ar import CustomAllReduce

        try:
            car = CustomAllReduce(self.group, capacity_mb=4.0)
        except RuntimeError:        # raised on every rank alike (the constructor agrees first)
            return None
        return car if car.enabled else None

    def query_payload(self, q: torch.Tensor) -> "np.ndarray":
        """The query block as host bytes for the replica's step channel (fp32 [n, dim]): the
        followers receive it inside the search command instead of through a broadcast."""
        return q.detach().to(torch.float32).reshape(-1, self.dim).cpu().contiguous().numpy()

    def queries_from_payload(self, n: int, payload) -> torch.Tensor:
        return torch.from_numpy(payload).view(torch.float32).view(n, self.dim).to(self.local.device)

    def search_side(self, payload, n: int, k: int, wait: bool = True):
        """A search whose query block every rank holds as host bytes (``query_payload``, sent in
        the step-channel command), run start to finish on the index's own stream: nothing on
        the engine's stream waits for it and it does not wait for the engine's in-flight step.
        ``wait``: return (scores, ids) on the host (the driver); else return None at once (a
        follower joins the collective and moves on)."""
        if self._stream is None:
            v, i = self.search(self.queries_from_payload(n, payload), k, have_queries=True)
            return (v.cpu(), i.cpu()) if wait else None
        with torch.cuda.stream(self._stream):
            v, i = self.search(self.queries_from_payload(n, payload), k, have_queries=True)
            if not wait:
                return None
            out = (v.cpu(), i.cpu())   # synchronises this stream only
        return out

    @torch.inference_mode()
    def search(self, q: torch.Tensor, k: int, src: int = 0,
               have_queries: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
        """Top-``k`` over every shard (collective over the group). ``have_queries``: every rank
        already holds ``q`` (it travelled in the step-channel command, ``query_payload``), so no
        broadcast is needed; otherwise rank ``src``'s block is broadcast first (CC7).

        Each rank's (score, id) list is packed into one int32 row per query — the k fp32 score
        bit patterns, then the k int64 ids as 2k words — and gathered in ONE collective (CC8):
        the index's own IPC all-gather kernel (ranks read each other's staging buffers over
        xGMI; no host round trip), else one process-group all-gather. The world x k candidates
        are merged by the top-k kernel (K15)."""
        if q.dim() == 1:
            q = q.unsqueeze(0)
        if self.world == 1:
            return self.local.search(q, k)
        t0 = time.perf_counter()
        if have_queries:
            qd = q.to(self.local.device, torch.float32).contiguous()
        else:
            qd = q.to(self.comm_dev, torch.float32).contiguous()
            dist.broadcast(qd, src=src, group=self.group)
            self.stats["broadcasts"] += 1
        vals, ids = self.local.search(qd.to(self.local.device), k)
        nq = qd.shape[0]
        kk = vals.shape[1]
        if kk < k:  # pad a short shard
            vals = torch.cat([vals, torch.full((nq, k - kk), float("-inf"), device=vals.device)], 1)
            ids = torch.cat([ids, torch.full((nq, k - kk), -1, dtype=torch.int64, device=ids.device)], 1)
        width = -(-3 * k // 4) * 4              # k scores + 2k id words, padded to 16-B rows
        # int32 words throughout, so no float path ever touches the id bits (a -1 id is a NaN
        # pattern as fp32)
        packed = torch.zeros(nq, width, dtype=torch.int32, device=vals.device)
        packed[:, :k] = vals.float().contiguous().view(torch.int32)
        packed[:, k:3 * k] = ids.to(torch.int64).contiguous().view(torch.int32)
        car = self._car if packed.is_cuda else None
        if car is not None and car.gather_eligible(packed):
            g = car.all_gather(packed)                                   # [nq, world * width]
            self.stats["ipc_gathers"] += 1
        else:
            parts = [torch.empty(nq, width, dtype=torch.int32, device=self.comm_dev) for _ in range(self.world)]
            dist.all_gather(parts, packed.to(self.comm_dev), group=self.group)
            g = torch.cat(parts, 1).to(self.local.device)
            self.stats["pg_gathers"] += 1
        g = g.view(nq, self.world, width)
        cv = g[:, :, :k].contiguous().view(torch.float32).reshape(nq, self.world * k).contiguous()
        ci = g[:, :, k:3 * k].contiguous().view(torch.int64).reshape(nq, self.world * k).contiguous()
        if cv.is_cuda:
            mv = torch.empty(nq, k, dtype=torch.float32, device=cv.device)
            mi = torch.empty(nq, k, dtype=torch.int64, device=cv.device)
            ops.kernels().topk(cv, ci, cv.shape[1], k, mv, mi)
        else:
            mv, pos = torch.topk(cv, k, dim=1)
            mi = torch.gather(ci, 1, pos)
        self.stats["searches"] += 1
        self.stats["host_s"] += time.perf_counter() - t0
        return mv, mi
