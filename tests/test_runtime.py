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
