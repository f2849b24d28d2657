"""IVF-Flat index (SURVEY.md §2.B N4 / kernel K14): the Milvus ``GPU_IVF_FLAT`` the
reference configures (nlist 64, nprobe 16 — RetrievalAugmentedGeneration/common/
configuration.py:38-47, utils.py:198-203).

* training: k-means on the GPU — assignment is the MFMA ``score`` kernel + exact top-1
  (``topk`` kernel) against the centroids, centroid update is a scatter-add;
* storage: vectors re-ordered by list into one contiguous bf16 slab with per-list offsets,
  so a probe scans contiguous HBM;
* search: coarse top-nprobe over centroids (batched over queries), then ONE launch of the
  fused score + top-k kernel over (list, query-chunk) work items: the (query, probe) pairs
  are grouped by list on the device, each probed list is streamed in place (no gather, no
  per-query loop, no host sync) once for every query probing it, and a final k-merge picks
  each query's top-k from its nprobe lists' candidates (``ops.ivf_search_topk``).

Flat search of a batch of queries reads the whole index once for the batch; IVF reads
nprobe/nlist of it per query — so IVF wins for small batches / latency, flat for big batches.
"""
from __future__ import annotations

import json
import os
from pathlib import Path
from typing import Optional, Tuple

import torch

from .. import ops


def kmeans(X: torch.Tensor, k: int, iters: int = 10, seed: int = 0, metric: str = "cosine") -> torch.Tensor:
    """k-means (spherical for cosine/ip) over bf16 rows X [n, d]; returns fp32 centroids [k, d]."""
    n = X.shape[0]
    g = torch.Generator(device="cpu").manual_seed(seed)
    C = X[torch.randperm(n, generator=g)[:k].to(X.device)].float()
    for _ in range(iters):
        a = assign(X, C, metric)
        sums = torch.zeros_like(C).index_add_(0, a, X.float())
        cnt = torch.bincount(a, minlength=k).float().unsqueeze(1)
        empty = cnt.squeeze(1) == 0
        C = torch.where(empty.unsqueeze(1), C, sums / cnt.clamp_min(1))
        if metric in ("cosine", "ip"):
            C = C / C.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    return C


def assign(X: torch.Tensor, C: torch.Tensor, metric: str = "cosine", chunk: int = 1 << 18) -> torch.Tensor:
    """Nearest centroid of every row (MFMA score kernel with centroids as the 'queries')."""
    Cb = C.to(X.dtype).contiguous()
    bias = -ops.row_sqnorm(Cb) if metric == "l2" else None
    out = []
    for s in range(0, X.shape[0], chunk):
        xs = X[s:s + chunk].contiguous()
        # rows of xs are the queries: S[i, c] = <x_i, c> (- |c|^2/2 via bias for l2)
        S = ops.score(xs, Cb, None if bias is None else bias * 0.5, 1.0)
        out.append(ops.topk(S, 1)[1][:, 0])
    return torch.cat(out)


class IVFFlatIndex:
    def __init__(self, dim: int, nlist: int = 64, nprobe: int = 16, metric: str = "cosine",
                 device: Optional[str] = None, dtype=torch.bfloat16):
        self.dim, self.nlist, self.nprobe, self.metric, self.dtype = dim, nlist, nprobe, metric, dtype
        self.device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        self.centroids: Optional[torch.Tensor] = None
        self.X = torch.zeros(0, dim, dtype=dtype, device=self.device)
        self.ids = torch.zeros(0, dtype=torch.int64, device=self.device)
        self.bias = torch.zeros(0, dtype=torch.float32, device=self.device)
        self.offsets = torch.zeros(nlist + 1, dtype=torch.int64)
        self._pending = []  # vectors added before training
        self._n_live = 0    # live (non-tombstoned) rows of the slab, kept on the host
        self._ranges = None  # device (list_beg, list_end) of the slab, rebuilt after adds

    def __len__(self):
        return self._n_live + sum(v.shape[0] for v, _ in self._pending)

    def _list_ranges(self):
        if self._ranges is None:
            off = self.offsets.to(self.device)
            self._ranges = (off[:-1].contiguous(), off[1:].contiguous(),
                            int((self.offsets[1:] - self.offsets[:-1]).max().item()) if self.nlist else 0)
        return self._ranges

    def _prep(self, v: torch.Tensor) -> torch.Tensor:
        v = v.to(self.device, torch.float32)
        if self.metric == "cosine":
            v = v / v.norm(dim=-1, keepdim=True).clamp_min(1e-12)
        return v

    @property
    def is_trained(self) -> bool:
        return self.centroids is not None

    def train(self, vecs: torch.Tensor, iters: int = 10, seed: int = 0):
        X = self._prep(vecs).to(self.dtype)
        k = min(self.nlist, X.shape[0])
        self.nlist = k
        self.centroids = kmeans(X, k, iters, seed, self.metric)
        self.offsets = torch.zeros(k + 1, dtype=torch.int64)
        pend, self._pending = self._pending, []
        for v, i in pend:
            self.add(v, i)

    def add(self, vecs: torch.Tensor, ids: torch.Tensor) -> None:
        if not self.is_trained:
            self._pending.append((vecs, ids))
            if sum(v.shape[0] for v, _ in self._pending) >= 39 * self.nlist:
                allv = torch.cat([self._prep(v) for v, _ in self._pending])
                self.train(allv)
            return
        X = self._prep(vecs).to(self.dtype)
        a = assign(X, self.centroids, self.metric)
        # merge into the list-sorted slab
        cur_list = torch.repeat_interleave(torch.arange(self.nlist), self.offsets[1:] - self.offsets[:-1]).to(self.device)
        allX = torch.cat([self.X, X])
        allI = torch.cat([self.ids, ids.to(self.device, torch.int64)])
        allB = torch.cat([self.bias, (-ops.row_sqnorm(X)) if self.metric == "l2" else torch.zeros(X.shape[0], device=self.device)])
        lists = torch.cat([cur_list, a])
        order = torch.argsort(lists, stable=True)
        self.X, self.ids, self.bias = allX[order].contiguous(), allI[order], allB[order]
        cnt = torch.bincount(lists, minlength=self.nlist).cpu()
        self.offsets = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(cnt, 0)])
        self._n_live += X.shape[0]
        self._ranges = None

    def _ensure_trained(self):
        """Train on whatever was added so far (k-means wants ~39 points per list, so adds
        are buffered until then; a search / save / remove forces training earlier)."""
        if not self.is_trained and self._pending:
            allv = torch.cat([self._prep(v) for v, _ in self._pending])
            self.train(allv)

    def remove(self, ids) -> int:
        self._ensure_trained()
        ids_t = torch.as_tensor(list(ids) if not torch.is_tensor(ids) else ids, dtype=torch.int64, device=self.device)
        hit = torch.isin(self.ids, ids_t) & torch.isfinite(self.bias)
        self.bias[hit] = float("-inf")
        n = int(hit.sum().item())
        self._n_live -= n
        return n

    @torch.inference_mode()
    def search(self, q: torch.Tensor, k: int, nprobe: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        if q.dim() == 1:
            q = q.unsqueeze(0)
        q = self._prep(q)
        nq = q.shape[0]
        self._ensure_trained()
        if not self.is_trained:
            return (torch.empty(nq, 0, device=self.device), torch.empty(nq, 0, dtype=torch.int64, device=self.device))
        nprobe = min(nprobe or self.nprobe, self.nlist)
        qb = q.to(self.dtype).contiguous()
        if self.X.shape[0] == 0 or k <= 0:
            return (torch.full((nq, max(k, 0)), float("-inf"), device=self.device),
                    torch.full((nq, max(k, 0)), -1, dtype=torch.int64, device=self.device))
        # coarse quantiser: top-nprobe centroids per query (MFMA score + top-k kernels)
        cS = ops.score(qb, self.centroids.to(self.dtype).contiguous(), None, 1.0)
        _, probes = ops.topk(cS, nprobe)
        beg, end, max_rows = self._list_ranges()
        scale = 2.0 if self.metric == "l2" else 1.0
        kmax = 64 if not ops._gpu(self.X) else ops.kernels().score_topk_kmax(min(nq, 64))
        if k <= kmax:
            vals, rows = ops.ivf_search_topk(qb, self.X, self.bias, scale, probes, beg, end, max_rows, k)
        else:   # beyond the fused kernel's register lists: per-query reference scan
            from ..ops import reference
            vals, rows = reference.ivf_search_topk(qb, self.X, self.bias, scale, probes, beg, end, k)
        if self.metric == "l2":
            vals = vals - q.float().pow(2).sum(-1, keepdim=True)
        ok = torch.isfinite(vals) & (rows >= 0)
        out_ids = torch.where(ok, self.ids[rows.clamp_min(0)], torch.full_like(rows, -1))
        return vals, out_ids

    def save(self, path: str):
        from safetensors.torch import save_file

        self._ensure_trained()
        p = Path(path)
        p.mkdir(parents=True, exist_ok=True)
        t = {"X": self.X.cpu(), "ids": self.ids.cpu(), "bias": self.bias.cpu(), "offsets": self.offsets}
        if self.centroids is not None:
            t["centroids"] = self.centroids.cpu()
        tmp = p / "vectors.safetensors.tmp"
        save_file(t, str(tmp))
        os.replace(tmp, p / "vectors.safetensors")
        (p / "index.json").write_text(json.dumps({"kind": "ivf_flat", "dim": self.dim, "nlist": self.nlist,
                                                   "nprobe": self.nprobe, "metric": self.metric}))

    @classmethod
    def load(cls, path: str, device: Optional[str] = None) -> "IVFFlatIndex":
        from safetensors.torch import load_file

        p = Path(path)
        m = json.loads((p / "index.json").read_text())
        t = load_file(str(p / "vectors.safetensors"))
        idx = cls(m["dim"], m["nlist"], m["nprobe"], m["metric"], device)
        idx.X, idx.ids, idx.bias = t["X"].to(idx.device), t["ids"].to(idx.device), t["bias"].to(idx.device)
        idx.offsets = t["offsets"]
        idx._n_live = int(torch.isfinite(t["bias"]).sum())
        if "centroids" in t:
            idx.centroids = t["centroids"].to(idx.device)
        return idx
