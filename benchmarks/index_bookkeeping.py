"""Index bookkeeping rate: a /documents-style ingestion of N chunk embeddings into the flat
index in batches (the embedding itself excluded: vectors are precomputed), then deletes.

Compares the native batched bookkeeping of ``index/flat.py`` (``_rt.IdMap`` + one tombstone
scatter per call) with the round-2 form (a Python dict updated per id, one device sync per
deleted row), kept here as ``LegacyFlatIndex`` for the before/after number.

    python benchmarks/index_bookkeeping.py --n 1000000 --batch 1024 --device cuda
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nv_genai_amd.index.flat import FlatIndex  # noqa: E402


class LegacyFlatIndex(FlatIndex):
    """Round-2 bookkeeping: per-id dict updates and a per-row ``.item()`` tombstone check."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self._id2row = {}

    def add(self, vecs, ids=None):
        vecs = self._prep(vecs)
        m = vecs.shape[0]
        ids = ids.to(torch.int64).cpu()
        if self.n + m > self.capacity:
            cap = self.capacity
            while cap < self.n + m:
                cap *= 2
            self._alloc(cap)
        r0 = self.n
        self.X[r0:r0 + m] = vecs.to(self.dtype)
        self.bias[r0:r0 + m] = 0.0
        self.ids[r0:r0 + m] = ids.to(self.device)
        for j, i in enumerate(ids.tolist()):
            if i in self._id2row:
                self._delete_row(self._id2row[i])
            self._id2row[i] = r0 + j
        self.n += m
        return ids

    def _delete_row(self, r):
        if self.bias[r].item() != float("-inf"):
            self.bias[r] = float("-inf")
            self.n_deleted += 1

    def remove(self, ids):
        cnt = 0
        for i in ids.tolist():
            r = self._id2row.pop(int(i), None)
            if r is not None:
                self._delete_row(r)
                cnt += 1
        return cnt


def run(cls, X, batch, n_del, dev):
    idx = cls(X.shape[1], "cosine", dev, capacity=X.shape[0])
    sync = (lambda: torch.cuda.synchronize()) if str(dev).startswith("cuda") else (lambda: None)
    sync()
    t0 = time.perf_counter()
    for s in range(0, X.shape[0], batch):
        idx.add(X[s:s + batch], torch.arange(s, min(s + batch, X.shape[0])))
    sync()
    t_add = time.perf_counter() - t0
    dels = torch.randperm(X.shape[0], generator=torch.Generator().manual_seed(0))[:n_del]
    t0 = time.perf_counter()
    removed = 0
    for s in range(0, n_del, 1000):
        removed += idx.remove(dels[s:s + 1000])
    sync()
    t_del = time.perf_counter() - t0
    assert removed == n_del and len(idx) == X.shape[0] - n_del
    return {"add_s": round(t_add, 3), "adds_per_s": round(X.shape[0] / t_add), "remove_s": round(t_del, 3),
            "removes_per_s": round(n_del / t_del)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--deletes", type=int, default=100_000)
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    g = torch.Generator(device=a.device).manual_seed(1)
    X = torch.randn(a.n, a.dim, device=a.device, generator=g).to(torch.bfloat16)
    # a short warm-up of both (allocator, first-touch pages, kernels), then the timed runs
    for cls in (FlatIndex, LegacyFlatIndex):
        run(cls, X[: min(a.n, 20 * a.batch)], a.batch, min(a.deletes, 1000), a.device)
    res = {"n": a.n, "dim": a.dim, "batch": a.batch, "deletes": a.deletes, "device": a.device,
           "legacy_dict": run(LegacyFlatIndex, X, a.batch, a.deletes, a.device),
           "native": run(FlatIndex, X, a.batch, a.deletes, a.device)}
    res["add_speedup"] = round(res["legacy_dict"]["add_s"] / res["native"]["add_s"], 2)
    res["remove_speedup"] = round(res["legacy_dict"]["remove_s"] / res["native"]["remove_s"], 2)
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
