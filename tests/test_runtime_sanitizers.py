"""ASan + UBSan build of the native host runtime (_rt: paged-KV block manager, continuous-
batching scheduler, BM25 index, splitters, HNSW graph index, step channel), driven by a randomized stress workload in a
child interpreter (the reference has no sanitizer coverage at all).

The instrumented module is built into a temp dir (the in-tree _rt stays uninstrumented) and
loaded with libasan preloaded ahead of anything already in LD_PRELOAD; any ASan report or
UBSan "runtime error" fails the test (-fno-sanitize-recover makes UB fatal).
"""
import os
import shutil
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STRESS = textwrap.dedent(r'''
    import importlib.util, random, sys
    import numpy as np
    spec = importlib.util.spec_from_file_location("_rt", sys.argv[1])
    rt = importlib.util.module_from_spec(spec); spec.loader.exec_module(rt)
    rng = random.Random(0)

    # block manager: random alloc / release / prefix register / lookup, incl. error paths
    bm = rt.BlockManager(64, 16, True)
    live = []
    for it in range(20000):
        op = rng.random()
        if op < 0.45 and bm.num_free() > 0:
            b = bm.alloc(); live.append(b)
            if rng.random() < 0.5:
                bm.register_full(b, rng.randrange(1 << 60))
        elif op < 0.85 and live:
            bm.release(live.pop(rng.randrange(len(live))))
        else:
            b = bm.lookup(rng.randrange(1 << 60))
            if b >= 0: live.append(b)
    for bad in (-1, 64, 10 ** 6):
        try:
            bm.release(bad)
        except (RuntimeError, ValueError, IndexError):
            pass

    # scheduler: random arrivals, chunked prefill, mixed steps, finishes, preemption pressure
    T, S, MB = 512, 16, 64
    s = rt.Scheduler(48, 16, S, T, 1024, True)
    s.set_mixed_prefill_tokens(128)
    bufs = (np.zeros(T, np.int32), np.zeros(T, np.int32), np.zeros(T, np.int32), np.zeros(S + 1, np.int32),
            np.zeros(S, np.int32), np.zeros((S, MB), np.int32), np.zeros(S, np.int64), np.zeros(S, np.int32))
    nxt, active = 1, set()
    for step in range(3000):
        if rng.random() < 0.3 and len(active) < 40:
            n = rng.randrange(1, 300)
            base = rng.randrange(4)  # shared prefixes exercise the prefix cache
            s.add(nxt, [base * 1000 + (i % 97) for i in range(n)], rng.randrange(1, 40))
            active.add(nxt); nxt += 1
        if not s.has_work():
            continue
        kind, n, ntok = s.schedule(*bufs)
        sids = [int(x) for x in bufs[6][:n]]
        smp = [int(x) for x in bufs[7][:n]]
        for sid, sm in zip(sids, smp):
            if sm and sid in active:
                s.append_token(sid, rng.randrange(50000))
                if rng.random() < 0.05 or s.num_generated(sid) > 30:
                    s.finish(sid); active.discard(sid)
    for sid in list(active):
        s.finish(sid)
    assert s.used_blocks() == 0 or not s.has_work()

    # BM25 + splitters
    idx = rt.BM25Index(1.2, 0.75)
    words = ["alpha", "beta", "gamma", "delta", "epsilon", "zeta", "eta", "theta", "x" * 300, ""]
    for d in range(3000):
        idx.add(d, " ".join(rng.choice(words) for _ in range(rng.randrange(0, 60))))
    for d in range(0, 3000, 7):
        idx.remove(d)
    for _ in range(200):
        idx.search(" ".join(rng.choice(words) for _ in range(rng.randrange(0, 6))), rng.randrange(1, 50))
    for n in (0, 1, 5, 510, 10000):
        rt.token_windows(n, 508, 200)
    text = "".join(rng.choice(["a", "b", " ", "\n", "\n\n", ". "]) for _ in range(20000))
    rt.char_split(text, 1000, 100, ["\n\n", "\n", " ", ""])
    rt.char_split("", 10, 0, ["\n"])

    # HNSW: interleaved adds / deletes / threaded searches, save + load, error paths
    import os, tempfile
    nr = np.random.default_rng(0)
    for metric in ("l2", "ip", "cosine"):
        h = rt.HNSW(24, metric, 6, 32, 16, 7)
        nid = 0
        for rnd in range(6):
            n = int(nr.integers(1, 400))
            h.add(nr.standard_normal((n, 24)).astype(np.float32), np.arange(nid, nid + n, dtype=np.int64))
            nid += n
            h.remove([int(x) for x in nr.integers(0, nid, 50)])
            h.search(nr.standard_normal((int(nr.integers(1, 40)), 24)).astype(np.float32), int(nr.integers(0, 20)),
                     int(nr.integers(0, 64)), int(nr.integers(1, 5)))
        f = os.path.join(tempfile.mkdtemp(), "g.hnsw")
        h.save(f)
        rt.HNSW.load(f).search(np.zeros((3, 24), np.float32), 5, 0, 2)
        for bad in (lambda: h.add(np.zeros((1, 24), np.float32), np.array([1], np.int64)) if len(h) else None,
                    lambda: h.search(np.zeros((1, 3), np.float32), 2, 0, 1),
                    lambda: rt.HNSW.load(f + ".missing")):
            try:
                bad()
            except (RuntimeError, ValueError):
                pass
    # step channel: ring wrap with varying message sizes, every error path, close
    name = f"/nga_asan_{os.getpid()}"
    w = rt.ShmChannel(name, True, 3, 512, 1, 0, 30.0)
    rd = rt.ShmChannel(name, False, 0, 0, 0, 0, 30.0)
    buf = np.empty(512, np.uint8)
    for i in range(2000):
        msg = nr.integers(0, 255, int(nr.integers(1, 513)), dtype=np.uint8)
        assert w.write(msg, 5.0) == 1
        n = rd.read(buf, 5.0)
        assert n == msg.size and bytes(buf[:n]) == msg.tobytes()
    for bad in (lambda: w.write(np.zeros(513, np.uint8), 1.0), lambda: rd.write(np.zeros(1, np.uint8), 1.0),
                lambda: w.read(buf, 1.0), lambda: rd.read(np.empty(4, np.uint8), 0.01),
                lambda: rt.ShmChannel(name, False, 0, 0, 0, 5, 30.0), lambda: rt.ShmChannel("bad", True, 2, 64, 1, 0, 1.0)):
        try:
            bad()
        except (RuntimeError, ValueError):
            pass
    assert rd.read(buf, 0.01) == -1
    w.unlink(); w.close()
    assert rd.read(buf, 1.0) == -2
    rd.stats(); w.stats()
    del w, rd
    print("STRESS_OK")
''')


@pytest.mark.timeout(600)
def test_runtime_under_asan_ubsan(tmp_path):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    libasan = subprocess.run(["g++", "-print-file-name=libasan.so"], capture_output=True,
                             text=True).stdout.strip()
    if not os.path.isabs(libasan) or not os.path.exists(libasan):
        pytest.skip("libasan not available")
    sys.path.insert(0, ROOT)
    from nv_genai_amd import _build

    san = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
           "-fno-omit-frame-pointer", "-g"]
    so = _build.build_runtime(force=True, out_dir=tmp_path, extra_flags=san)
    script = tmp_path / "stress.py"
    script.write_text(STRESS)
    env = dict(os.environ)
    # libstdc++ right after libasan: python itself does not link it, and ASan's
    # __cxa_throw interceptor must resolve the real one when _rt throws
    libstdcxx = subprocess.run(["g++", "-print-file-name=libstdc++.so.6"], capture_output=True,
                               text=True).stdout.strip()
    env["LD_PRELOAD"] = " ".join(p for p in (libasan, libstdcxx, os.environ.get("LD_PRELOAD", "")) if p)
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1"
    r = subprocess.run([sys.executable, str(script), str(so)], capture_output=True, text=True,
                       env=env, timeout=500)
    report = r.stdout[-3000:] + r.stderr[-6000:]
    assert r.returncode == 0, report
    assert "STRESS_OK" in r.stdout, report
    assert "AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr, report


TSAN_WORKLOAD = textwrap.dedent(r'''
    import importlib.util, sys
    import numpy as np
    spec = importlib.util.spec_from_file_location("_rt", sys.argv[1])
    rt = importlib.util.module_from_spec(spec); spec.loader.exec_module(rt)
    rng = np.random.default_rng(0)
    # multi-threaded HNSW batch linking (striped link-list locks) and threaded batch search
    for metric in ("l2", "cosine"):
        h = rt.HNSW(16, metric, 8, 48, 32, 1)
        h.add(rng.standard_normal((2500, 16)).astype(np.float32), np.arange(2500, dtype=np.int64), 8)
        h.add(rng.standard_normal((1500, 16)).astype(np.float32), np.arange(2500, 4000, dtype=np.int64), 8)
        h.remove(list(range(0, 4000, 5)))
        h.search(rng.standard_normal((400, 16)).astype(np.float32), 10, 64, 8)
    # the step channel: one writer and two readers on three threads (the GIL is released in
    # write / read), each object with its heartbeat thread; futex sleeps and wake-ups
    import os, threading, time
    name = f"/nga_tsan_{os.getpid()}"
    w = rt.ShmChannel(name, True, 4, 256, 2, 0, 30.0)
    rds = [rt.ShmChannel(name, False, 0, 0, 0, i, 30.0) for i in range(2)]
    w.unlink()
    got = [[], []]
    def reader(i):
        buf = np.empty(256, np.uint8)
        for _ in range(3000):
            n = rds[i].read(buf, 30.0)
            assert n == 8, n
            got[i].append(int(buf[:8].view(np.int64)[0]))
    ts = [threading.Thread(target=reader, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for s in range(3000):
        if s % 500 == 0:
            time.sleep(0.05)    # readers fall asleep on the futex now and then
        assert w.write(np.array([s], np.int64), 30.0) == 1
    for t in ts:
        t.join()
    assert got[0] == got[1] == list(range(3000))
    rds[0].stats(); w.stats()
    w.close()
    del rds, w
    print("TSAN_OK")
''')


@pytest.mark.timeout(600)
def test_hnsw_parallel_build_under_tsan(tmp_path):
    """ThreadSanitizer build of _rt driving its multi-threaded native code: the HNSW parallel
    build / search and the step channel (writer, readers and heartbeat threads)."""
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    libtsan = subprocess.run(["g++", "-print-file-name=libtsan.so"], capture_output=True,
                             text=True).stdout.strip()
    if not os.path.isabs(libtsan) or not os.path.exists(libtsan):
        pytest.skip("libtsan not available")
    sys.path.insert(0, ROOT)
    from nv_genai_amd import _build

    so = _build.build_runtime(force=True, out_dir=tmp_path, extra_flags=["-fsanitize=thread", "-g", "-O1"])
    script = tmp_path / "tsan.py"
    script.write_text(TSAN_WORKLOAD)
    env = dict(os.environ)
    env["LD_PRELOAD"] = " ".join(p for p in (libtsan, os.environ.get("LD_PRELOAD", "")) if p)
    env["TSAN_OPTIONS"] = "report_signal_unsafe=0"
    r = subprocess.run([sys.executable, str(script), str(so)], capture_output=True, text=True,
                       env=env, timeout=500)
    report = r.stdout[-3000:] + r.stderr[-6000:]
    assert r.returncode == 0, report
    assert "TSAN_OK" in r.stdout, report
    assert "ThreadSanitizer" not in r.stderr, report
