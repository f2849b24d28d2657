"""HNSW index build / search rate and recall on the host (csrc/runtime/hnsw.cpp), with the
reference's streaming-ingest index parameters (kafka_config.yaml:112-122: HNSW, L2, M 8,
efConstruction 64, 384-d MiniLM embeddings). Recall@k is against exact search. Synthetic
clustered vectors (embeddings are clustered, not uniform). Prints one JSON line."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50000)
    ap.add_argument("--dim", type=int, default=384)
    ap.add_argument("--queries", type=int, default=1000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--M", type=int, default=8)
    ap.add_argument("--ef-construction", type=int, default=64)
    ap.add_argument("--ef", default="16,32,64,128")
    ap.add_argument("--metric", default="l2")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from nv_genai_amd.index.hnsw import HNSWIndex

    rng = np.random.default_rng(0)
    cent = rng.standard_normal((256, a.dim)).astype(np.float32)
    X = (cent[rng.integers(0, 256, a.n)] + 0.5 * rng.standard_normal((a.n, a.dim))).astype(np.float32)
    Q = (cent[rng.integers(0, 256, a.queries)] + 0.5 * rng.standard_normal((a.queries, a.dim))).astype(np.float32)
    idx = HNSWIndex(a.dim, a.metric, M=a.M, ef_construction=a.ef_construction, threads=a.threads)
    t0 = time.perf_counter()
    idx.add(X, np.arange(a.n))
    build = time.perf_counter() - t0
    # exact top-k (squared L2 / dot) in blocks
    exact = []
    for s in range(0, a.queries, 256):
        q = Q[s:s + 256]
        sc = -((q ** 2).sum(1)[:, None] - 2 * q @ X.T + (X ** 2).sum(1)[None]) if a.metric == "l2" else q @ X.T
        exact.append(np.argpartition(-sc, a.k, axis=1)[:, :a.k])
    exact = np.concatenate(exact)
    res = []
    for ef in [int(e) for e in a.ef.split(",")]:
        t0 = time.perf_counter()
        _, ids = idx.search(Q, a.k, ef=ef)
        dt = time.perf_counter() - t0
        t1 = time.perf_counter()
        for i in range(min(200, a.queries)):
            idx.search(Q[i], a.k, ef=ef)
        single = (time.perf_counter() - t1) / min(200, a.queries)
        rec = float(np.mean([len(set(g.tolist()) & set(e.tolist())) / a.k for g, e in zip(ids.numpy(), exact)]))
        res.append({"ef": ef, "recall_at_k": round(rec, 4), "batch_qps": round(a.queries / dt, 1),
                    "single_query_us": round(1e6 * single, 1)})
    line = {"metric": "HNSW host index", "n": a.n, "dim": a.dim, "M": a.M, "ef_construction": a.ef_construction,
            "index_metric": a.metric, "k": a.k, "threads": a.threads, "build_s": round(build, 2),
            "build_vectors_per_s": round(a.n / build, 1), "search": res,
            "data": "synthetic clustered vectors (256 centres)"}
    s = json.dumps(line)
    print(s, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
