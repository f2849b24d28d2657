"""Native host runtime (_rt): block manager, continuous-batching scheduler, BM25, splitters."""
import numpy as np
import pytest

from nv_genai_amd._native import rt


def _bufs(T=256, S=8, MB=16):
    return (np.zeros(T, np.int32), np.zeros(T, np.int32), np.zeros(T, np.int32), np.zeros(S + 1, np.int32),
            np.zeros(S, np.int32), np.zeros((S, MB), np.int32), np.zeros(S, np.int64), np.zeros(S, np.int32))


def test_block_manager_refcount_and_prefix_cache():
    bm = rt.BlockManager(4, 16, True)
    a = bm.alloc()
    bm.register_full(a, 123)
    bm.release(a)
    assert bm.num_free() == 4  # cached but evictable
    assert bm.lookup(123) == a  # revived from the LRU
    assert bm.num_free() == 3
    bm.release(a)
    blocks = [bm.alloc() for _ in range(4)]  # forces eviction of the cached block
    assert sorted(blocks) == [0, 1, 2, 3]
    assert bm.lookup(123) == -1
    with pytest.raises(RuntimeError):
        bm.release(99)


def test_scheduler_prefill_then_decode_and_chunking():
    s = rt.Scheduler(32, 16, 8, 40, 256, True)
    s.add(1, list(range(1, 31)), 5)   # 30 tokens
    s.add(2, list(range(100, 150)), 5)  # 50 tokens
    b = _bufs()
    kind, n, ntok = s.schedule(*b)
    ids, pos, sl, cu, ctx, bt, sid, smp = b
    assert kind == 1 and ntok == 40  # token budget: seq1 whole + 10 of seq2
    assert list(sid[:n]) == [1, 2] and list(cu[: n + 1]) == [0, 30, 40]
    assert list(smp[:n]) == [1, 0]  # seq2's chunk is not its last
    assert list(pos[:30]) == list(range(30)) and list(ids[30:40]) == list(range(100, 110))
    s.append_token(1, 7)
    kind, n, ntok = s.schedule(*b)  # continue seq2's prefill (priority over decode)
    assert kind == 1 and list(sid[:n]) == [2] and ntok == 40 and ctx[0] == 50 and smp[0] == 1
    s.append_token(2, 8)
    kind, n, ntok = s.schedule(*b)
    assert kind == 2 and n == 2 and list(ids[:2]) == [7, 8] and list(pos[:2]) == [30, 50]
    assert list(ctx[:2]) == [31, 51]
    # slots are consistent with the block table
    for i in range(2):
        p = pos[i]
        assert sl[i] == bt[i, p // 16] * 16 + p % 16
    s.finish(1)
    s.finish(2)
    assert not s.has_work() and s.used_blocks() == 0 or s.free_blocks() == 32


def test_scheduler_prefix_cache_hit_and_preemption():
    s = rt.Scheduler(8, 16, 8, 256, 256, True)
    prompt = list(range(1, 50))  # 49 tokens -> 3 full blocks reusable (keep >= 1 to compute)
    s.add(1, prompt, 2)
    b = _bufs()
    s.schedule(*b)
    s.append_token(1, 5)
    s.finish(1)
    s.add(2, prompt, 2)
    kind, n, ntok = s.schedule(*b)
    assert kind == 1 and ntok == 49 - 48 and s.cached_prefix(2) == 48
    assert s.prefix_hits() == 3
    s.finish(2)
    # preemption: 2 seqs, tiny cache, decode growth forces the later one out
    s2 = rt.Scheduler(4, 16, 8, 256, 256, False)
    s2.add(1, list(range(32)), 40)
    s2.add(2, list(range(32)), 40)
    s2.schedule(*b)  # both admitted? each needs 2 blocks -> 4 blocks total
    for _ in range(3):
        for sid_ in (1, 2):
            try:
                s2.append_token(sid_, 1)
            except Exception:
                pass
        kind, n, ntok = s2.schedule(*b)
    assert s2.preemptions() >= 1


def test_scheduler_token_alignment_leaves_no_short_tail():
    """Mixed steps round their token count down to the alignment by shortening the last prefill
    chunk, but not when that would leave its prompt a tail shorter than one alignment unit (the
    old rule then fed such a tail 256 - nd tokens a step). 6 decode rows + a 13-token prompt at
    alignment 8 run as one 19-token step; a 40-token prompt under a 26-token budget beside 7
    decode rows is cut to 25 (32 tokens, its 15-token rest >= 8), and the rest then runs whole
    (22 tokens: aligning to 16 would leave a 6-token tail)."""
    s = rt.Scheduler(64, 16, 8, 256, 256, False)
    s.set_mixed_prefill_tokens(64)
    s.set_token_alignment(8)
    b = _bufs()
    for i in range(6):
        s.add(i + 1, [10 + i] * 4, 8)
    kind, n, ntok = s.schedule(*b)
    assert kind == 1 and ntok == 24
    for i in range(6):
        s.append_token(i + 1, 1)
    s.add(9, list(range(1, 14)), 8)
    kind, n, ntok = s.schedule(*b)
    assert kind == 3 and n == 7 and ntok == 19 and s.last_num_decode() == 6
    ids, pos, sl, cu, ctx, bt, sid, smp = b
    assert sid[6] == 9 and smp[6] == 1 and ctx[6] == 13
    for i in range(6):
        s.append_token(i + 1, 1)
    s.append_token(9, 1)
    s.set_mixed_prefill_tokens(26)
    s.add(10, list(range(1, 41)), 8)
    kind, n, ntok = s.schedule(*b)
    assert kind == 3 and ntok == 32 and s.last_num_decode() == 7   # 7 decode + 25, aligned to 32
    for i in list(range(1, 7)) + [9]:
        s.append_token(i, 1)
    kind, n, ntok = s.schedule(*b)
    assert kind == 3 and ntok == 7 + 15                             # the 15-token rest, kept whole


def test_bm25_ranking_and_delete():
    b = rt.BM25Index()
    b.add(1, "the mi355x gpu has 288 gb of hbm3e memory")
    b.add(2, "bananas are yellow fruit")
    b.add(3, "memory bandwidth of hbm is high")
    r = b.search("hbm memory", 3)
    assert [d for d, _ in r][:2] == [1, 3] or [d for d, _ in r][:2] == [3, 1]
    assert 2 not in [d for d, _ in r]
    b.remove(1)
    assert [d for d, _ in b.search("hbm memory", 3)] == [3]
    assert len(b) == 2


def test_token_windows_and_char_split():
    assert rt.token_windows(10, 4, 1) == [(0, 4), (3, 7), (6, 10)]
    assert rt.token_windows(3, 8, 2) == [(0, 3)]
    chunks = rt.char_split("a" * 50 + "\n\n" + "b" * 50, 60, 0)
    assert chunks == ["a" * 50, "b" * 50]
    long = " ".join(f"w{i}" for i in range(200))
    cs = rt.char_split(long, 100, 20)
    assert all(len(c) <= 100 for c in cs) and len(cs) > 5


def test_idmap_matches_dict_under_random_ops():
    """Native id -> row map (csrc/runtime/idmap.cpp) against a Python dict through random
    batched adds (with re-adds and in-batch duplicates), removes, lookups and rebuilds."""
    import numpy as np

    from nv_genai_amd._native import rt

    rng = np.random.default_rng(0)
    m, ref = rt.IdMap(), {}
    row = 0
    for step in range(300):
        op = rng.integers(0, 3)
        if op == 0:
            ids = rng.integers(-50, 5000, size=int(rng.integers(1, 200)))
            disp = m.add(ids, row)
            want = []
            for j, i in enumerate(ids.tolist()):
                if i in ref:
                    want.append(ref[i])
                ref[i] = row + j
            row += len(ids)
            assert sorted(disp.tolist()) == sorted(want)
        elif op == 1:
            ids = rng.integers(-50, 5000, size=int(rng.integers(1, 300)))
            got = m.remove(ids)
            want = []
            for i in ids.tolist():
                if i in ref:
                    want.append(ref.pop(i))
            assert sorted(got.tolist()) == sorted(want)
        else:
            q = rng.integers(-60, 5100, size=100)
            assert m.rows(q).tolist() == [ref.get(i, -1) for i in q.tolist()]
        assert len(m) == len(ref)
    keys = np.array(sorted(ref), dtype=np.int64)
    live = (rng.random(len(keys)) < 0.7).astype(np.uint8)
    m.rebuild(keys, live)
    assert len(m) == int(live.sum())
    assert m.rows(keys).tolist() == [j if live[j] else -1 for j in range(len(keys))]
    m.add_range(100_000, 8, 1000, 7)
    assert m.rows(np.array([100_000, 100_008, 107_992, 100_001])).tolist() == [7, 8, 1006, -1]
    assert m.max_id() == 107_992


def test_flat_index_batched_bookkeeping():
    """FlatIndex add / re-add / remove / compact / save-load keep ids and live counts right
    with the native map (no per-id Python loop, one tombstone scatter per call)."""
    import torch

    from nv_genai_amd.index.flat import FlatIndex

    g = torch.Generator().manual_seed(0)
    X = torch.randn(3000, 32, generator=g)
    idx = FlatIndex(32, "cosine", "cpu", capacity=16)
    idx.add(X[:2000], torch.arange(2000) * 2)
    assert len(idx) == 2000
    idx.add(X[2000:2100], torch.arange(100) * 2)           # re-add 100 ids: old rows tombstoned
    assert len(idx) == 2000 and idx.n_deleted == 100
    s, i = idx.search(X[2000:2005], 1)
    assert i[:, 0].tolist() == [0, 2, 4, 6, 8]               # the new vectors answer for the ids
    assert idx.remove(torch.arange(0, 400, 2)) == 200 and len(idx) == 1800
    assert idx.remove([0, 2, 123456]) == 0
    auto = idx.add(X[2100:2110])                              # fresh ids continue after the max id
    assert auto.tolist() == list(range(3999, 3999 + 10))
    idx.compact()
    assert idx.n == len(idx) == 1810 and idx.n_deleted == 0
    s2, i2 = idx.search(X[2100:2103], 1)
    assert i2[:, 0].tolist() == [3999, 4000, 4001]
