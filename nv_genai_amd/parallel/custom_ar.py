"""Custom all-reduce for tensor-parallel decode: direct reads of IPC-mapped peer buffers
over xGMI (``csrc/kernels/custom_ar.hip``), with RCCL for everything it does not cover.

Where the reference gets this: TensorRT-LLM's ``enable_custom_all_reduce`` knob inside NIM
(experimental/fm-asr-streaming-rag/nim/configs/mistral-7b.yaml:36; SURVEY.md §2.D CC1/CC2,
§2.F). Llama-3-70B at TP=8 issues 160 all-reduces per generated token, each only
16 KiB x batch: RCCL's ring pays W-1 serial hops on one xGMI link each; here every rank
reads all 7 peers at once and a call is one (one-shot) or two (two-shot) cross-GPU flag
round trips plus the data time.

Construction is collective over the group: every rank allocates its uncached
Signal+staging block, the IPC handles are exchanged with ``all_gather_object`` and every
rank maps its peers. A start-up self-test compares the result against the process group's
own all-reduce (and checks the kernel's barrier-timeout flag) and all ranks agree on the
outcome; on any failure the object disables itself and callers fall back to RCCL.
"""
from __future__ import annotations

import logging
import os
from typing import Optional

import torch
import torch.distributed as dist

log = logging.getLogger(__name__)

ALGO_AUTO, ALGO_ONE_SHOT, ALGO_TWO_SHOT = 0, 1, 2
TWO_SHOT_THRESHOLD_BYTES = 512 * 1024   # the kernel's default (custom_ar.h)
MAX_BLOCKS = 80                          # kArMaxBlocks (custom_ar.h): the grid cap per call
# per staging buffer (x2 for the call-parity double buffer, uncached HBM): the largest message
# a step graph may hold — a 4,352-token mixed step of a hidden-8,192 model (71 MB bf16) and
# 256 rows of an 8B model's half vocabulary at TP=2 (66 MB fp32 logits)
DEFAULT_CAPACITY_MB = 80


def choose_algo(nbytes: int, world: int, threshold: int = TWO_SHOT_THRESHOLD_BYTES) -> int:
    """One-shot (every rank reads all W-1 peers' full message: one flag round trip, W-1
    times the bytes per link) below ``threshold``; two-shot (reduce-scatter of 1/W slices +
    all-gather: two round trips, 2/W of the bytes per link) above it. At W = 2 the two-shot
    saves nothing, so it is one-shot at every size."""
    return ALGO_TWO_SHOT if world > 2 and nbytes > threshold else ALGO_ONE_SHOT


class CustomAllReduce:
    def __init__(self, group=None, capacity_mb: float = 64.0, timeout_s: float = 5.0,
                 two_shot_threshold_kb: Optional[float] = None, self_test: bool = True):
        from ..ops import kernels

        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        cap = int(capacity_mb * 2 ** 20) // 128 * 128
        self.capacity = cap
        self.fused_norm_max_bytes = 1 << 20
        self.two_shot_threshold = (int(two_shot_threshold_kb * 1024) if two_shot_threshold_kb is not None
                                   else TWO_SHOT_THRESHOLD_BYTES)
        self.algo_counts = {ALGO_ONE_SHOT: 0, ALGO_TWO_SHOT: 0}
        self.gather_count = 0
        self.enabled = False
        self.impl = None
        # every stage ends with an agreement among the ranks, so a failure on one rank
        # never leaves the others waiting in a collective
        handle, err = b"", None
        try:
            self.impl = kernels().CustomAllReduce(self.rank, self.world, cap, float(timeout_s))
            self.impl.set_two_shot_threshold(self.two_shot_threshold)
            handle = self.impl.handle()
        except Exception as e:  # noqa: BLE001
            err = e
        if not self._agree(err is None):
            raise RuntimeError(f"custom all-reduce: allocation/export failed on some rank ({err!r})")
        handles = [None] * self.world
        dist.all_gather_object(handles, handle, group=group)
        try:
            self.impl.open(handles)
        except Exception as e:  # noqa: BLE001
            err = e
        if not self._agree(err is None):
            raise RuntimeError(f"custom all-reduce: mapping peer buffers failed on some rank ({err!r})")
        # ranks sharing one device (one-GPU rehearsals): every rank's spinning blocks must be
        # resident at once, so each call gets a share of the grid cap
        self.ranks_per_device = self._ranks_per_device()
        blocks = os.environ.get("NGA_CUSTOM_AR_BLOCKS")
        if blocks:
            self.impl.set_max_blocks(int(blocks))
        elif self.ranks_per_device > 1:
            self.impl.set_max_blocks(max(4, MAX_BLOCKS // self.ranks_per_device))
        self.max_blocks = int(self.impl.max_blocks())
        self.enabled = True
        if self_test:
            self.enabled = self._self_test()

    # ------------------------------------------------------------------ API
    def eligible(self, x: torch.Tensor) -> bool:
        nbytes = x.numel() * x.element_size()
        return (self.enabled and x.is_cuda and x.is_contiguous()
                and x.dtype in (torch.bfloat16, torch.float32)
                and 0 < nbytes <= self.capacity and nbytes % 16 == 0
                and x.data_ptr() % 16 == 0)

    def all_reduce(self, x: torch.Tensor, out: Optional[torch.Tensor] = None,
                   algo: int = ALGO_AUTO) -> torch.Tensor:
        """Sum of ``x`` over the group (in place unless ``out`` is given). ``ALGO_AUTO`` is
        resolved here (:func:`choose_algo`), so the kernel always receives an explicit one."""
        if out is None:
            out = x
        if algo == ALGO_AUTO:
            algo = choose_algo(x.numel() * x.element_size(), self.world, self.two_shot_threshold)
        self.algo_counts[algo] = self.algo_counts.get(algo, 0) + 1
        self.impl.all_reduce(x, out, algo)
        return out

    def fused_norm_eligible(self, x: torch.Tensor) -> bool:
        """The one-shot all-reduce + residual add + RMSNorm kernel takes bf16 [rows, H]
        messages up to ``fused_norm_max_bytes`` (above that the two-shot all-reduce plus a
        separate add+norm moves fewer bytes over xGMI)."""
        return (self.eligible(x) and x.dtype == torch.bfloat16 and x.dim() == 2
                and x.shape[1] % 8 == 0 and x.shape[1] <= 16384
                and x.numel() * 2 <= self.fused_norm_max_bytes)

    def all_reduce_add_rmsnorm(self, x: torch.Tensor, resid: torch.Tensor, w: torch.Tensor,
                               eps: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """resid += all_reduce(x) (in place); returns rmsnorm(resid) * w."""
        if out is None:
            out = torch.empty_like(resid)
        self.impl.all_reduce_add_rmsnorm(x, resid, w, out, float(eps))
        return out

    def gather_eligible(self, x: torch.Tensor) -> bool:
        """The IPC all-gather along the last dim takes contiguous 2-D device tensors whose rows
        are whole 16-B packets and whose shard fits the staging buffer."""
        return (self.enabled and x.is_cuda and x.is_contiguous() and x.dim() == 2
                and (x.shape[1] * x.element_size()) % 16 == 0 and x.data_ptr() % 16 == 0
                and 0 < x.numel() * x.element_size() <= self.capacity)

    def all_gather(self, x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """[rows, cols] per rank -> [rows, world * cols], rank r's shard in columns
        [r * cols, (r + 1) * cols) (the vocab-parallel LM head's logits). Capture-safe."""
        if out is None:
            out = torch.empty(x.shape[0], self.world * x.shape[1], dtype=x.dtype, device=x.device)
        self.gather_count += 1
        self.impl.all_gather(x, out)
        return out

    def error(self) -> int:
        """0, or the code of the first barrier that timed out (1 one-shot, 2 / 3 two-shot
        start / mid, 4 all-reduce + RMSNorm, 5 all-gather)."""
        return int(self.impl.error())

    def _ranks_per_device(self) -> int:
        """How many ranks of the group run on this rank's physical device (host, PCI id)."""
        from ..parallel.step_channel import _host_key

        pr = torch.cuda.get_device_properties(torch.cuda.current_device())
        key = (_host_key(), getattr(pr, "pci_domain_id", None), getattr(pr, "pci_bus_id", None),
               getattr(pr, "pci_device_id", None), str(getattr(pr, "uuid", "")))
        keys = [None] * self.world
        dist.all_gather_object(keys, key, group=self.group)
        return sum(k == key for k in keys)

    def _agree(self, ok: bool) -> bool:
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
        if dist.get_backend(self.group) == "nccl":
            flag = flag.to(torch.device("cuda", torch.cuda.current_device()))
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
        return bool(flag.item())

    # ------------------------------------------------------------------ self-test
    def _reference_sum(self, x: torch.Tensor) -> torch.Tensor:
        backend = dist.get_backend(self.group)
        y = x.float().clone() if backend == "nccl" else x.float().cpu()
        dist.all_reduce(y, group=self.group)
        return y.to(x.device)

    def _reference_gather(self, x: torch.Tensor) -> torch.Tensor:
        backend = dist.get_backend(self.group)
        y = x.contiguous() if backend == "nccl" else x.cpu()
        parts = [torch.empty_like(y) for _ in range(self.world)]
        dist.all_gather(parts, y, group=self.group)
        return torch.cat(parts, dim=1).to(x.device)

    def _self_test(self) -> bool:
        ok = True
        dev = torch.device("cuda", torch.cuda.current_device())
        try:
            dist.barrier(group=self.group)
            for n, algo in ((4096, ALGO_ONE_SHOT), (1 << 20, ALGO_TWO_SHOT), (1 << 20, ALGO_AUTO)):
                g = torch.Generator(device="cpu").manual_seed(1000 + self.rank)
                x = torch.randn(n, generator=g).to(dev, torch.bfloat16)
                ref = self._reference_sum(x)
                got = self.all_reduce(x.clone(), algo=algo)
                torch.cuda.synchronize(dev)
                # no early exit: every rank must issue the same collectives
                ok = ok and not self.error() and torch.allclose(got.float(), ref, atol=0.05, rtol=0.02)
            # the all-gather: fp32 shards with a rank-dependent pattern, compared bit for bit
            g = torch.Generator(device="cpu").manual_seed(2000 + self.rank)
            shard = torch.randn(3, 68, generator=g).to(dev)
            want = self._reference_gather(shard)
            got = self.all_gather(shard)
            torch.cuda.synchronize(dev)
            ok = ok and not self.error() and torch.equal(got, want)
        except Exception as e:  # noqa: BLE001 - any failure means "use RCCL"
            log.warning("custom all-reduce self-test raised: %r", e)
            ok = False
        ok = self._agree(ok)
        if not ok:
            log.warning("custom all-reduce disabled (self-test failed); TP all-reduces use RCCL")
        return ok


_STATUS = {"state": "not requested"}
_LAST = None


def status() -> dict:
    """Outcome of this process's last :func:`maybe_create` (for run records): ``state`` is
    "not requested", "off" (world / device / NGA_CUSTOM_AR), "failed" (construction raised),
    "self-test failed" (RCCL takes every all-reduce) or "enabled"; with the one-/two-shot call
    counts of the Python entry point (calls recorded into a hipGraph count once, at capture)."""
    s = dict(_STATUS)
    if _LAST is not None:
        s["max_blocks"] = _LAST.max_blocks
        s["ranks_per_device"] = _LAST.ranks_per_device
        try:   # the kernels' sticky barrier-timeout flag (0: every call met its peers in time)
            s["timeout_flag"] = _LAST.error()
        except Exception as e:  # noqa: BLE001
            s["timeout_flag"] = repr(e)[:80]
        s["algo_counts"] = {"one_shot": _LAST.algo_counts.get(ALGO_ONE_SHOT, 0),
                            "two_shot": _LAST.algo_counts.get(ALGO_TWO_SHOT, 0)}
    return s


def maybe_create(group, world: int) -> Optional[CustomAllReduce]:
    """The TP group's custom all-reduce, or None when it does not apply (CPU, world 1 or
    > 8, ``NGA_CUSTOM_AR=0``). Collective: every rank of ``group`` must call it."""
    global _STATUS, _LAST
    _STATUS = {"state": "off", "world": world}
    if world <= 1 or world > 8 or not torch.cuda.is_available():
        return None
    if os.environ.get("NGA_CUSTOM_AR", "1") == "0":
        return None
    try:
        car = CustomAllReduce(group, capacity_mb=float(os.environ.get("NGA_CUSTOM_AR_MB", str(DEFAULT_CAPACITY_MB))))
    except Exception as e:  # noqa: BLE001
        log.warning("custom all-reduce unavailable (%r); TP all-reduces use RCCL", e)
        _STATUS = {"state": "failed", "world": world, "error": repr(e)[:200]}
        return None
    _STATUS = {"state": "enabled" if car.enabled else "self-test failed", "world": world,
               "self_test_passed": bool(car.enabled)}
    _LAST = car if car.enabled else None
    return _LAST
