"""Driver -> follower channel for the step layouts of a model-parallel replica (CC5).

Every step of a TP / PP replica is scheduled once, on its driver (tp rank 0, stage 0), and
each follower rank must run the same forward on the same layout. The layout is host data
(token ids, positions, cache slots, block tables, sampling parameters, and the rows whose
input ids the previous step is still producing on the device). Two transports:

* :class:`ShmStepChannel` — all ranks of the replica on one node (the TP=8 agent, the TP=2
  one-GPU rehearsal): a ring of shared-memory slots (``_rt.ShmChannel``, C++). Publishing is a
  memcpy plus a release store, so the driver never waits on its GPU to publish and followers
  start launching step k + 1 while step k still runs — the pipelined TP engine.
* :class:`DistStepChannel` — anything else: a length-prefixed broadcast over the replica's
  process group (RCCL or gloo). Correct everywhere, but over RCCL the host payload is staged
  through the driver's current stream, so the engine keeps such replicas unpipelined.

The reference's TP engine hides this inside TensorRT-LLM's in-flight batching with
``tensor_para_size`` (experimental/fm-asr-streaming-rag/nim/configs/mistral-7b.yaml:26-39).
"""
from __future__ import annotations

import os
import socket
import uuid
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from .._native import rt
from .dist import ParallelContext

# one slot must hold the largest step message; the ring depth bounds how far the driver may
# run ahead of the slowest follower (the engine itself keeps at most one step in flight)
DEFAULT_SLOTS = 4


def _env_float(name: str, default: float) -> float:
    v = os.environ.get(name)
    return float(v) if v not in (None, "") else default


def step_timeout_s() -> float:
    """Hard limit on one channel wait (``NGA_STEP_TIMEOUT_S``; default -1 = none). An idle
    replica publishes no steps, so followers wait for the next one indefinitely; a dead peer
    is found by its heartbeat instead (:func:`step_liveness_s`)."""
    return _env_float("NGA_STEP_TIMEOUT_S", -1.0)


def step_liveness_s() -> float:
    """A peer whose heartbeat (stamped every 100 ms by a native thread of its channel) is this
    old is dead (``NGA_STEP_LIVENESS_S``, default 30 s; <= 0 turns the check off)."""
    return _env_float("NGA_STEP_LIVENESS_S", 30.0)


class PeerDiedError(RuntimeError):
    """The peer a channel wait depends on stopped its heartbeat (process gone or frozen)."""


class StepChannel:
    pipelined = False   # True: publishing never waits for the driver's GPU

    def send(self, msg: np.ndarray) -> None:
        raise NotImplementedError

    def recv(self) -> np.ndarray:
        raise NotImplementedError

    def stats(self) -> dict:
        return {}

    def close(self) -> None:
        pass


class ShmStepChannel(StepChannel):
    pipelined = True

    def __init__(self, pctx: ParallelContext, slot_bytes: int, nslots: int = DEFAULT_SLOTS,
                 timeout_s: Optional[float] = None, liveness_s: Optional[float] = None):
        self.p = pctx
        self.timeout = float(step_timeout_s() if timeout_s is None else timeout_s)
        liveness = float(step_liveness_s() if liveness_s is None else liveness_s)
        self.slot_bytes = int(slot_bytes)
        driver = pctx.tp_rank == 0 and pctx.pp_rank == 0
        name = None
        err = None
        if driver:
            name = f"/nga_step_{os.getpid()}_{uuid.uuid4().hex[:12]}"
            try:
                self.ch = rt.ShmChannel(name, True, nslots, self.slot_bytes, pctx.mp_size - 1, 0, liveness)
            except Exception as e:  # noqa: BLE001
                err, name = e, None
        obj = [name]
        dist.broadcast_object_list(obj, src=pctx.mp_src, group=pctx.mp_group)
        name = obj[0]
        if name is None:
            raise RuntimeError(f"shm step channel: the driver could not create its segment ({err!r})")
        ok = True
        if not driver:
            # reader index: this rank's position among the replica's followers
            local = pctx.rank - pctx.mp_src
            try:
                self.ch = rt.ShmChannel(name, False, 0, 0, 0, local - 1, liveness)
                self._buf = np.empty(self.ch.slot_bytes(), dtype=np.uint8)
            except Exception as e:  # noqa: BLE001 - e.g. ranks on different hosts after all
                ok, err = False, e
        # every follower attached (or not): agree, then drop the name so nothing is left in
        # /dev/shm on a crash
        oks = [None] * pctx.mp_size
        dist.all_gather_object(oks, ok, group=pctx.mp_group)
        if driver:
            self.ch.unlink()
        if not all(oks):
            if driver:
                self.ch.close()
            raise ShmAttachError(f"shm step channel: {oks.count(False)} follower(s) could not attach"
                                 + (f" ({err!r})" if not ok else ""))
        self.driver = driver

    def send(self, msg: np.ndarray) -> None:
        rc = self.ch.write(np.ascontiguousarray(msg), self.timeout)
        if rc == -3:
            raise PeerDiedError("step channel: a follower stopped its heartbeat")
        if rc == -2:
            raise RuntimeError("step channel closed")
        if rc != 1:
            raise TimeoutError("step channel: followers stopped consuming")

    def recv(self) -> np.ndarray:
        n = self.ch.read(self._buf, self.timeout)
        if n == -2:
            raise RuntimeError("step channel closed by the driver")
        if n == -3:
            raise PeerDiedError("step channel: the driver stopped its heartbeat")
        if n < 0:
            raise TimeoutError("step channel: no step from the driver")
        return self._buf[:n]

    def stats(self) -> dict:
        """Follower: publish -> receipt latency percentiles (µs) over the last messages and how
        its waits ended (spin / yield / futex sleep); driver: its own waits for ring space."""
        return dict(self.ch.stats())

    def close(self) -> None:
        self.ch.close()


class ShmAttachError(RuntimeError):
    """A follower could not open the driver's segment (raised on every rank of the replica)."""


class DistStepChannel(StepChannel):
    """Length-prefixed broadcast over the replica's process group (device tensors on RCCL)."""

    def __init__(self, pctx: ParallelContext, slot_bytes: int):
        self.p = pctx
        self.slot_bytes = int(slot_bytes)
        self.dev = pctx.device if pctx.backend == "nccl" else torch.device("cpu")

    def _bcast(self, t: torch.Tensor) -> torch.Tensor:
        x = t.to(self.dev)
        dist.broadcast(x, src=self.p.mp_src, group=self.p.mp_group)
        return x

    def send(self, msg: np.ndarray) -> None:
        b = torch.from_numpy(np.ascontiguousarray(msg).view(np.uint8))
        self._bcast(torch.tensor([b.numel()], dtype=torch.int64))
        self._bcast(b)

    def recv(self) -> np.ndarray:
        n = int(self._bcast(torch.zeros(1, dtype=torch.int64)).cpu()[0])
        return self._bcast(torch.empty(n, dtype=torch.uint8)).cpu().numpy()


def _host_key() -> tuple:
    """(hostname, kernel boot id): containers on one host share the boot id, and two hosts that
    happen to carry the same container hostname do not."""
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            boot = f.read().strip()
    except OSError:
        boot = ""
    return socket.gethostname(), boot


def same_host(pctx: ParallelContext) -> bool:
    """Every rank of this rank's replica runs on this node (collective over the replica)."""
    keys = [None] * pctx.mp_size
    dist.all_gather_object(keys, _host_key(), group=pctx.mp_group)
    return len(set(keys)) == 1


def create(pctx: ParallelContext, slot_bytes: int, transport: Optional[str] = None) -> StepChannel:
    """The replica's step channel (collective over its ranks). ``transport``: "shm", "dist" or
    None (shm when the replica is on one node; ``NGA_STEP_CHANNEL`` overrides)."""
    transport = transport or os.environ.get("NGA_STEP_CHANNEL") or None
    if transport is None:
        transport = "shm" if same_host(pctx) else "dist"
    if transport == "shm":
        try:
            return ShmStepChannel(pctx, slot_bytes)
        except ShmAttachError:
            if os.environ.get("NGA_STEP_CHANNEL") == "shm":
                raise          # asked for explicitly: fail loudly
            return DistStepChannel(pctx, slot_bytes)
    if transport == "dist":
        return DistStepChannel(pctx, slot_bytes)
    raise ValueError(f"step channel transport must be shm or dist, not {transport!r}")
