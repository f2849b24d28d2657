"""CPU / NUMA placement of one-process-per-GPU ranks.

On a two-socket 8-GPU node each GPU hangs off one socket's PCIe root. A rank whose host
threads (step loop, tokenizer pool, pinned-memory copies, the chain server's event loop) float
onto the other socket pays the inter-socket hop on every H2D / D2H transfer and shares last
level cache with another GPU's rank. The reference pins services to GPUs per container
(``deploy/compose/compose.env:1-75``, ``docker-compose-nim-ms.yaml:15-21`` device ids); here each
rank binds itself, before it touches the GPU, to the cores of its GPU's NUMA node, split evenly
among the local ranks that share that node.

The GPU of a local rank is found WITHOUT initialising HIP (the HIP runtime must not start
before the affinity is set, or its own threads keep the old mask): the KFD topology
(``/sys/class/kfd/kfd/topology/nodes/*/properties``: the GPU nodes in HIP's enumeration order,
each with its PCI ``domain`` / ``location_id``) filtered by ``HIP_VISIBLE_DEVICES`` /
``ROCR_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES``, then the PCI device's ``numa_node`` and the
node's ``cpulist``. Every sysfs path hangs off ``root`` so tests can use a fake tree.
"""
from __future__ import annotations

import logging
import os
from dataclasses import dataclass, field
from typing import List, Optional

log = logging.getLogger(__name__)


@dataclass
class GpuInfo:
    index: int            # HIP device index among the visible devices
    pci: str              # dddd:bb:dd.f
    numa_node: int        # -1: unknown / single node


@dataclass
class Placement:
    local_rank: int
    gpu: Optional[GpuInfo] = None
    numa_node: int = -1
    cpus: List[int] = field(default_factory=list)
    physical_cores: int = 0          # whole cores given to the rank (every SMT sibling included)
    l3_domains: List[str] = field(default_factory=list)   # L3 domains (shared_cpu_list) it touches
    whole_l3: bool = False           # every touched L3 domain belongs to this rank alone
    applied: bool = False
    reason: str = ""

    def record(self) -> dict:
        return {"numa_node": self.numa_node, "cpu_affinity": _ranges(self.cpus),
                "physical_cores": self.physical_cores, "l3_domains": self.l3_domains,
                "whole_l3": self.whole_l3,
                "pci_bus_id_sysfs": self.gpu.pci if self.gpu else None,
                "affinity_applied": self.applied, **({"affinity_note": self.reason} if self.reason else {})}


def parse_cpulist(s: str) -> List[int]:
    out: List[int] = []
    for part in s.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def _ranges(cpus: List[int]) -> str:
    if not cpus:
        return ""
    cpus = sorted(cpus)
    parts, lo, prev = [], cpus[0], cpus[0]
    for c in cpus[1:] + [None]:
        if c is not None and c == prev + 1:
            prev = c
            continue
        parts.append(f"{lo}-{prev}" if prev > lo else str(lo))
        if c is not None:
            lo = prev = c
    return ",".join(parts)


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


def kfd_gpus(root: str = "/") -> List[GpuInfo]:
    """GPU nodes of the KFD topology in node order (HIP's device order), with PCI address and
    NUMA node; empty when there is no KFD (no GPU driver)."""
    base = os.path.join(root, "sys/class/kfd/kfd/topology/nodes")
    try:
        nodes = sorted(int(n) for n in os.listdir(base) if n.isdigit())
    except OSError:
        return []
    gpus: List[GpuInfo] = []
    for n in nodes:
        txt = _read(os.path.join(base, str(n), "properties"))
        if not txt:
            continue
        props = {}
        for line in txt.splitlines():
            kv = line.split()
            if len(kv) == 2 and kv[1].lstrip("-").isdigit():
                props[kv[0]] = int(kv[1])
        if props.get("simd_count", 0) <= 0 or props.get("cpu_cores_count", 0) > 0:
            continue   # a CPU node
        loc, dom = props.get("location_id", 0), props.get("domain", 0)
        pci = f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 0x7:x}"
        numa = _read(os.path.join(root, "sys/bus/pci/devices", pci, "numa_node"))
        gpus.append(GpuInfo(index=len(gpus), pci=pci, numa_node=int(numa) if numa and numa.strip() else -1))
    return gpus


def visible_gpus(root: str = "/", env=None) -> List[GpuInfo]:
    """The KFD GPUs after the runtime's visibility masks, re-indexed as HIP numbers them."""
    env = os.environ if env is None else env
    gpus = kfd_gpus(root)
    # ROCR's mask applies first (it hides agents from the HIP runtime); HIP then applies
    # HIP_VISIBLE_DEVICES, and CUDA_VISIBLE_DEVICES only when HIP's own variable is unset
    hip_var = "HIP_VISIBLE_DEVICES" if env.get("HIP_VISIBLE_DEVICES") else "CUDA_VISIBLE_DEVICES"
    for var in ("ROCR_VISIBLE_DEVICES", hip_var):
        v = env.get(var)
        if v is None or v == "":
            continue
        try:
            keep = [int(x) for x in v.split(",") if x.strip() != ""]
        except ValueError:   # UUID-style masks: leave the order alone
            continue
        gpus = [gpus[i] for i in keep if 0 <= i < len(gpus)]
    return [GpuInfo(index=i, pci=g.pci, numa_node=g.numa_node) for i, g in enumerate(gpus)]


@dataclass
class _Core:
    cpus: List[int]       # logical CPUs of one physical core (SMT siblings), allowed ones only
    l3: str               # the core's L3 domain (its shared_cpu_list; "" when unknown)


def cpu_topology(cpus: List[int], root: str = "/") -> List[_Core]:
    """Group logical CPUs into physical cores (``topology/thread_siblings_list``, else
    (``physical_package_id``, ``core_id``)) tagged with their L3 domain
    (``cache/index3/shared_cpu_list``), ordered by L3 domain and then by first CPU. A CPU with
    no topology in sysfs is a core of its own."""
    base = os.path.join(root, "sys/devices/system/cpu")
    want = set(cpus)
    cores: dict = {}
    for c in cpus:
        d = os.path.join(base, f"cpu{c}")
        sib = _read(os.path.join(d, "topology/thread_siblings_list"))
        if sib and sib.strip():
            key = ("sib", _ranges(parse_cpulist(sib)))
        else:
            pkg, cid = _read(os.path.join(d, "topology/physical_package_id")), _read(os.path.join(d, "topology/core_id"))
            key = ("id", pkg.strip(), cid.strip()) if pkg and cid else ("cpu", c)
        l3 = _read(os.path.join(d, "cache/index3/shared_cpu_list"))
        core = cores.setdefault(key, _Core(cpus=[], l3=_ranges(parse_cpulist(l3)) if l3 and l3.strip() else ""))
        if c in want:
            core.cpus.append(c)
    out = [k for k in cores.values() if k.cpus]
    l3_first = {}
    for k in out:
        l3_first[k.l3] = min(l3_first.get(k.l3, 1 << 30), min(k.cpus))
    out.sort(key=lambda k: (l3_first[k.l3], min(k.cpus)))
    return out


def split_cores(cores: List[_Core], k: int) -> List[List[_Core]]:
    """Split cores among ``k`` ranks: whole L3 domains per rank when there are at least ``k``
    of them (domains dealt out contiguously, balanced by core count), else contiguous runs of
    whole cores in L3 order, so no two ranks share a physical core and each rank's cores sit
    in as few L3 domains as possible."""
    if k <= 0 or not cores:
        return [[] for _ in range(max(k, 0))]
    domains: List[List[_Core]] = []
    for c in cores:
        if domains and domains[-1][0].l3 == c.l3:
            domains[-1].append(c)
        else:
            domains.append([c])
    if len(domains) >= k and all(d[0].l3 for d in domains):
        parts: List[List[_Core]] = [[] for _ in range(k)]
        total, acc, r = len(cores), 0, 0
        for i, d in enumerate(domains):
            # move on to the next rank once this one holds its share of cores, leaving at
            # least one domain for every rank still to come
            if parts[r] and r < k - 1 and (acc >= (r + 1) * total / k or len(domains) - i <= k - 1 - r):
                r += 1
            parts[r].extend(d)
            acc += len(d)
        return parts
    n = len(cores)
    if n < k:   # fewer cores than ranks: ranks share cores round-robin
        return [[cores[i % n]] for i in range(k)]
    return [cores[i * n // k:(i + 1) * n // k] for i in range(k)]


def plan(local_rank: int, local_world: int, root: str = "/", env=None,
         allowed: Optional[List[int]] = None) -> Placement:
    """Cores for ``local_rank``: its GPU's NUMA node's CPUs (intersected with the CPUs this
    process may use), split among the local ranks whose GPUs share that node in whole
    physical cores (all SMT siblings of a core go to one rank) and, where the node has at
    least one L3 domain per rank, in whole L3 domains."""
    pl = Placement(local_rank=local_rank)
    gpus = visible_gpus(root, env)
    if allowed is None:
        allowed = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else []
    if not gpus:
        pl.reason = "no KFD topology"
        return pl
    ng = len(gpus)
    gpu_of = [r % ng for r in range(local_world)]     # ranks share devices round-robin past ng
    g = gpus[gpu_of[local_rank]]
    pl.gpu, pl.numa_node = g, g.numa_node
    if g.numa_node < 0:
        pl.reason = "GPU has no NUMA node"
        return pl
    txt = _read(os.path.join(root, f"sys/devices/system/node/node{g.numa_node}/cpulist"))
    if not txt:
        pl.reason = "no cpulist for the NUMA node"
        return pl
    node_cpus = [c for c in parse_cpulist(txt) if c in set(allowed)] if allowed else parse_cpulist(txt)
    if not node_cpus:
        pl.reason = "the NUMA node's CPUs are outside this process's CPU set"
        return pl
    peers = [r for r in range(local_world) if gpus[gpu_of[r]].numa_node == g.numa_node]
    k, i = len(peers), peers.index(local_rank)
    parts = split_cores(cpu_topology(node_cpus, root), k)
    mine = parts[i]
    pl.cpus = sorted(c for core in mine for c in core.cpus)
    pl.physical_cores = len(mine)
    pl.l3_domains = sorted({core.l3 for core in mine if core.l3}, key=lambda t: parse_cpulist(t)[0])
    others = {core.l3 for j, p in enumerate(parts) if j != i for core in p}
    pl.whole_l3 = bool(pl.l3_domains) and not (set(pl.l3_domains) & others)
    return pl


def bind_local_rank(local_rank: int, local_world: int, root: str = "/", env=None) -> Placement:
    """Plan and apply (``sched_setaffinity``) this rank's placement; sizes the tokenizer
    (rayon) and OpenMP pools to it unless the environment already set them. Call before any
    HIP call. ``NGA_NUMA_BIND=0`` turns it off."""
    env = os.environ if env is None else env
    pl = plan(local_rank, local_world, root, env)
    if env.get("NGA_NUMA_BIND", "1") == "0":
        pl.reason = "NGA_NUMA_BIND=0"
        return pl
    if pl.cpus and hasattr(os, "sched_setaffinity"):
        try:
            os.sched_setaffinity(0, pl.cpus)
            pl.applied = True
            n = str(len(pl.cpus))
            env.setdefault("RAYON_NUM_THREADS", n)
            env.setdefault("OMP_NUM_THREADS", n)
        except OSError as e:
            pl.reason = f"sched_setaffinity failed: {e}"
    return pl
