"""In-process stack sampler for the serving processes (no py-spy in the image).

A daemon thread wakes every ``interval_s`` and records, for every other Python thread, the
innermost frame and a short stack (``sys._current_frames``). Per thread it counts samples in
which the thread was parked (selector / lock / queue / sleep waits) separately from those in
which it held or wanted the interpreter, so "the event loop is saturated" or "the engine thread
waits on the GIL" can be read off the output. The aggregate is written as JSON every
``dump_every_s`` (and at exit), so a server killed by its benchmark still leaves it.

Enabled by ``NGA_PY_SAMPLE_OUT=<path>`` in the chain server and the model server
(``NGA_PY_SAMPLE_MS`` = interval, default 20 ms). The sampler holds the GIL once per interval
for a few microseconds per live thread: at 5 ms with ~100 worker threads that perturbed the
chain server measurably, so sample sparsely and run longer.
"""
from __future__ import annotations

import atexit
import collections
import json
import os
import sys
import threading
import time
from typing import Dict, Optional

# leaf functions in which a thread is parked, not running Python
_IDLE = {"select", "poll", "epoll", "wait", "_wait_for_tstate_lock", "acquire", "get", "sleep",
         "accept", "recv", "recv_into", "readinto", "_worker", "wait_for", "run_forever", "_run_once",
         "synchronize", "join"}


def _where(f) -> str:
    c = f.f_code
    return f"{os.path.basename(c.co_filename)}:{c.co_name}:{f.f_lineno}"


class StackSampler:
    def __init__(self, path: str, interval_s: float = 0.005, dump_every_s: float = 20.0, depth: int = 8):
        self.path, self.interval_s, self.dump_every_s, self.depth = path, interval_s, dump_every_s, depth
        self.samples = 0
        self.per_thread: Dict[str, collections.Counter] = collections.defaultdict(collections.Counter)
        self.leaf: Dict[str, collections.Counter] = collections.defaultdict(collections.Counter)
        self.stacks: Dict[str, collections.Counter] = collections.defaultdict(collections.Counter)
        self._stop = threading.Event()
        self._lock = threading.Lock()    # one sample and one summary never interleave
        self._thread = threading.Thread(target=self._run, name="nga-stack-sampler", daemon=True)
        self.t0 = time.time()

    def start(self) -> "StackSampler":
        self._thread.start()
        atexit.register(self.stop)
        return self

    def stop(self) -> None:
        if not self._stop.is_set():
            self._stop.set()
            # the sampler thread may be inside a sample: let it finish before summarising
            if self._thread.is_alive() and self._thread is not threading.current_thread():
                self._thread.join(timeout=1.0)
            self.dump()

    def _run(self) -> None:
        me = threading.get_ident()
        last = time.monotonic()
        while not self._stop.wait(self.interval_s):
            names = {t.ident: t.name for t in threading.enumerate()}
            with self._lock:
                self._sample(me, names)
            if time.monotonic() - last > self.dump_every_s:
                last = time.monotonic()
                self.dump()

    def _sample(self, me: int, names: dict) -> None:
        for ident, frame in sys._current_frames().items():
            if ident == me:
                continue
            name = names.get(ident, str(ident))
            # thread pools: one bucket per pool, not per worker
            key = name.rstrip("0123456789_-") or name
            leaf = frame.f_code.co_name
            idle = leaf in _IDLE
            self.per_thread[key]["idle" if idle else "busy"] += 1
            if not idle:
                self.leaf[key][_where(frame)] += 1
                st, f = [], frame
                while f is not None and len(st) < self.depth:
                    st.append(_where(f))
                    f = f.f_back
                self.stacks[key][" <- ".join(st)] += 1
        self.samples += 1

    def summary(self, top: int = 25) -> dict:
        with self._lock:
            return self._summary(top)

    def _summary(self, top: int) -> dict:
        out = {"samples": self.samples, "interval_ms": self.interval_s * 1e3,
               "wall_s": round(time.time() - self.t0, 1), "threads": {}}
        for k, c in sorted(self.per_thread.items(), key=lambda kv: -kv[1]["busy"]):
            tot = c["busy"] + c["idle"]
            out["threads"][k] = {"busy_share": round(c["busy"] / max(1, tot), 4), "samples": tot,
                                 "top_leaf": self.leaf[k].most_common(top),
                                 "top_stacks": self.stacks[k].most_common(max(5, top // 3))}
        return out

    def dump(self) -> None:
        try:
            tmp = self.path + ".tmp"
            with open(tmp, "w") as f:
                json.dump(self.summary(), f, indent=1)
            os.replace(tmp, self.path)
        except (OSError, RuntimeError):   # unwritable path; a summary raced by interpreter exit
            pass


_ACTIVE: Optional[StackSampler] = None


def start_from_env(tag: str = "") -> Optional[StackSampler]:
    """Start the process's sampler when ``NGA_PY_SAMPLE_OUT`` names a file ({tag} and {pid}
    are substituted); idempotent."""
    global _ACTIVE
    path = os.environ.get("NGA_PY_SAMPLE_OUT")
    if not path or _ACTIVE is not None:
        return _ACTIVE
    path = path.replace("{tag}", tag or "proc").replace("{pid}", str(os.getpid()))
    _ACTIVE = StackSampler(path, float(os.environ.get("NGA_PY_SAMPLE_MS", "20")) / 1e3).start()
    return _ACTIVE
