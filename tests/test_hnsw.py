"""HNSW graph index (csrc/runtime/hnsw.cpp via index/hnsw.py): recall against exact search
for each metric, tombstone deletes, persistence, threaded batch search, the reference's
``index_conf`` mapping (kafka_config.yaml:109-125) and the VectorStore integration."""
import numpy as np
import pytest
import torch

from nv_genai_amd.index.hnsw import HNSWIndex
from nv_genai_amd.ingest.streaming import store_kwargs


def _exact(X, Q, k, metric):
    if metric == "l2":
        s = -((Q[:, None, :] - X[None]) ** 2).sum(-1)
    else:
        if metric == "cosine":
            X = X / np.linalg.norm(X, axis=1, keepdims=True)
            Q = Q / np.linalg.norm(Q, axis=1, keepdims=True)
        s = Q @ X.T
    return np.argsort(-s, axis=1)[:, :k], np.sort(s, axis=1)[:, ::-1][:, :k]


@pytest.mark.parametrize("metric,threads", [("l2", 1), ("ip", 4), ("cosine", 8), ("l2", 6)])
def test_recall_against_exact_search(metric, threads):
    rng = np.random.default_rng(0)
    X = rng.standard_normal((4000, 32)).astype(np.float32)
    Q = rng.standard_normal((100, 32)).astype(np.float32)
    idx = HNSWIndex(32, metric, M=16, ef_construction=200, ef=128, threads=threads)
    # two batches: the second links into a graph that already exists
    idx.add(torch.from_numpy(X[:1500]), torch.arange(1500) + 10)
    idx.add(torch.from_numpy(X[1500:]), torch.arange(1500, 4000) + 10)
    assert len(idx) == 4000
    s, i = idx.search(torch.from_numpy(Q), 10)
    ref_i, ref_s = _exact(X, Q, 10, metric)
    recall = np.mean([len(set(a) & set(b + 10)) / 10 for a, b in zip(i.numpy(), ref_i)])
    assert recall >= 0.95, recall
    # scores are the metric's similarity (-L2^2 / dot), sorted best first
    assert np.all(np.diff(s.numpy(), axis=1) <= 1e-5)
    hit = i.numpy()[:, 0] == ref_i[:, 0] + 10
    np.testing.assert_allclose(s.numpy()[hit, 0], ref_s[hit, 0], rtol=1e-4, atol=1e-4)


def test_delete_persist_threads_and_errors(tmp_path):
    rng = np.random.default_rng(1)
    X = rng.standard_normal((1500, 16)).astype(np.float32)
    idx = HNSWIndex(16, "l2", M=8, ef_construction=64, ef=64, threads=4)
    idx.add(X, np.arange(1500))
    gone = list(range(0, 1500, 3))
    assert idx.remove(gone) == len(gone)
    assert idx.remove(gone[:5]) == 0                       # already deleted
    assert len(idx) == 1000
    s, i = idx.search(X[:64], 5)
    assert not set(i.numpy().ravel().tolist()) & set(gone)
    # threaded batch == one query at a time
    for r in range(0, 64, 7):
        s1, i1 = idx.search(X[r], 5)
        assert i1.numpy()[0].tolist() == i.numpy()[r].tolist()
    idx.save(str(tmp_path))
    again = HNSWIndex.load(str(tmp_path))
    s2, i2 = again.search(X[:64], 5)
    assert torch.equal(i2, i) and torch.equal(s2, s) and len(again) == 1000
    with pytest.raises(Exception):
        idx.add(X[:1], np.array([1]))                       # duplicate live id
    with pytest.raises(Exception):
        idx.add(X[:2], np.array([5000, 5000]))              # duplicate inside a batch
    assert len(idx) == 1000
    idx.add(X[:1], np.array([5000]))                        # the failed batch left no trace
    assert len(idx) == 1001
    idx.remove([5000])
    with pytest.raises(Exception):
        idx.search(np.zeros((1, 15), np.float32), 3)        # wrong dim
    e = HNSWIndex(16, "l2")
    s, i = e.search(X[:2], 3)
    assert (i.numpy() == -1).all()


def test_reference_index_conf_mapping():
    vcfg = {"resource_schemas": {
        "vdb_kafka_scrape": {"index_conf": {"field_name": "embedding", "metric_type": "L2", "index_type": "HNSW",
                                            "params": {"M": 8, "efConstruction": 64}}},
        "gpu": {"index_conf": {"metric_type": "IP", "index_type": "GPU_IVF_FLAT", "params": {"nlist": 64}}},
        "plain": {}}}
    assert store_kwargs(vcfg, "vdb_kafka_scrape") == {"metric": "l2", "index_type": "hnsw", "hnsw_m": 8,
                                                      "hnsw_ef_construction": 64}
    assert store_kwargs(vcfg, "gpu") == {"metric": "ip", "index_type": "ivf_flat", "nlist": 64}
    assert store_kwargs(vcfg, "plain") == {} and store_kwargs({}, "x") == {}


def test_load_rejects_corrupt_graph(tmp_path):
    """A graph file whose neighbour ids, link counts or entry point do not fit the index is
    refused at load (search trusts the loaded graph without bounds checks)."""
    import shutil
    import struct

    rng = np.random.default_rng(2)
    n, d, M = 300, 8, 8
    X = rng.standard_normal((n, d)).astype(np.float32)
    idx = HNSWIndex(d, "l2", M=M, ef_construction=32, ef=32, threads=2)
    idx.add(X, np.arange(n))
    good = tmp_path / "good"
    idx.save(str(good))
    raw = (good / "graph.hnsw").read_bytes()
    l0 = 8 + 28 + 8 + n * d * 4 + n * 8 + n + n * 4      # start of the level-0 link lists
    hdr_entry = 8 + 5 * 4

    def corrupt(name, off, value):
        dst = tmp_path / name
        shutil.copytree(good, dst)
        b = bytearray(raw)
        b[off:off + 4] = struct.pack("<i", value)
        (dst / "graph.hnsw").write_bytes(bytes(b))
        return str(dst)

    for path in (corrupt("nbr", l0 + 4, 10 ** 6),            # node 0's first neighbour id
                 corrupt("cnt", l0, 2 * M + 5),               # node 0's level-0 link count
                 corrupt("entry", hdr_entry, n + 3)):          # entry point past the end
        with pytest.raises(Exception, match="corrupt"):
            HNSWIndex.load(path)
    s, i = HNSWIndex.load(str(good)).search(X[:4], 3)
    assert i.numpy()[:, 0].tolist() == [0, 1, 2, 3]


def test_flat_add_random_collision_leaves_index_unchanged():
    """add_random with ids that collide with existing ones raises before touching the slab or
    the id map (the map and the rows used to diverge)."""
    import pytest
    import torch

    from nv_genai_amd.index.flat import FlatIndex

    idx = FlatIndex(32, "cosine", "cpu", capacity=64)
    idx.add_random(10, seed=1)
    n0, X0 = idx.n, idx.X[:10].clone()
    with pytest.raises(ValueError):
        idx.add_random(5, seed=2, first_id=7)          # ids 7..11 overlap 0..9
    assert idx.n == n0 and torch.equal(idx.X[:10], X0)
    idx.add_random(5, seed=2)                           # the next free ids still work
    assert idx.n == 15
    v, r = idx.search(idx.X[12:13].float(), 1)
    assert int(r[0, 0]) == 12
