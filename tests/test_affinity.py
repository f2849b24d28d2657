"""NUMA placement of one-process-per-GPU ranks (utils/affinity.py) from a fake sysfs tree:
an 8-GPU, two-socket node (GPUs 0-3 on node 0, 4-7 on node 1), visibility masks, ranks that
share a node split its cores, and a process whose CPU set excludes the node."""
import os

import pytest

from nv_genai_amd.utils import affinity


def _node(root, n, props):
    d = root / "sys/class/kfd/kfd/topology/nodes" / str(n)
    d.mkdir(parents=True)
    (d / "properties").write_text("".join(f"{k} {v}\n" for k, v in props.items()))


def _tree(tmp_path):
    root = tmp_path
    # KFD: two CPU nodes first, then eight GPUs (bus 0x05, 0x15, ... ; HIP's order)
    _node(root, 0, {"cpu_cores_count": 48, "simd_count": 0})
    _node(root, 1, {"cpu_cores_count": 48, "simd_count": 0})
    for g in range(8):
        bus = 0x05 + 0x10 * g
        _node(root, 2 + g, {"cpu_cores_count": 0, "simd_count": 1024, "location_id": bus << 8, "domain": 0,
                            "gpu_id": 1000 + g})
        pci = root / "sys/bus/pci/devices" / f"0000:{bus:02x}:00.0"
        pci.mkdir(parents=True)
        (pci / "numa_node").write_text(f"{0 if g < 4 else 1}\n")
    for n, cpus in ((0, "0-47,96-143"), (1, "48-95,144-191")):
        d = root / f"sys/devices/system/node/node{n}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cpus + "\n")
    return str(root)


def test_cpulist_roundtrip():
    assert affinity.parse_cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]
    assert affinity._ranges([0, 1, 2, 3, 8, 10, 11]) == "0-3,8,10-11"


def test_eight_ranks_split_their_sockets(tmp_path):
    root = _tree(tmp_path)
    allowed = list(range(192))
    gpus = affinity.visible_gpus(root, env={})
    assert [g.pci for g in gpus][:2] == ["0000:05:00.0", "0000:15:00.0"] and len(gpus) == 8
    seen = set()
    for r in range(8):
        pl = affinity.plan(r, 8, root, env={}, allowed=allowed)
        node = 0 if r < 4 else 1
        assert pl.numa_node == node and pl.gpu.index == r
        assert len(pl.cpus) == 24                       # 96 node CPUs over 4 ranks
        node_cpus = set(affinity.parse_cpulist("0-47,96-143" if node == 0 else "48-95,144-191"))
        assert set(pl.cpus) <= node_cpus
        assert not (set(pl.cpus) & seen)                # disjoint between ranks
        seen |= set(pl.cpus)
        rec = pl.record()
        assert rec["numa_node"] == node and rec["cpu_affinity"]


def test_visibility_mask_and_foreign_cpuset(tmp_path):
    root = _tree(tmp_path)
    # the job sees GPUs 6 and 1 (in that order): local rank 0 is GPU 6 on node 1
    pl = affinity.plan(0, 2, root, env={"HIP_VISIBLE_DEVICES": "6,1"}, allowed=list(range(192)))
    assert pl.gpu.pci == "0000:65:00.0" and pl.numa_node == 1 and len(pl.cpus) == 96
    pl1 = affinity.plan(1, 2, root, env={"HIP_VISIBLE_DEVICES": "6,1"}, allowed=list(range(192)))
    assert pl1.numa_node == 0
    # a container limited to node 0's first cores: rank on node 1 is left unbound
    pl = affinity.plan(5, 8, root, env={}, allowed=list(range(8)))
    assert pl.cpus == [] and "outside" in pl.reason
    # no KFD: nothing to do
    assert affinity.plan(0, 2, str(tmp_path / "nothing"), env={}).reason == "no KFD topology"


def test_bind_applies_and_sizes_pools(tmp_path, monkeypatch):
    root = _tree(tmp_path)
    calls = []
    monkeypatch.setattr(os, "sched_setaffinity", lambda pid, cpus: calls.append(sorted(cpus)))
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(192)))
    env = {}
    pl = affinity.bind_local_rank(3, 8, root, env=env)
    assert pl.applied and calls == [pl.cpus] and env["RAYON_NUM_THREADS"] == "24"
    off = affinity.bind_local_rank(3, 8, root, env={"NGA_NUMA_BIND": "0"})
    assert not off.applied and len(calls) == 1


def test_doctor_report_on_this_host(tmp_path):
    """tools/doctor.py: the deployment report loads both native libraries, lists the code
    objects bundled in _C (gfx950) and the kernel-form registry, and reads gfx targets from a
    HIP binary's offload-bundle ids."""
    from nv_genai_amd.tools import doctor

    rep = doctor.collect()
    assert rep["native_C"] and rep["native_rt"], rep["problems"]
    assert rep["native_C_targets"] == ["gfx950"]
    assert set(rep["kernel_forms"]) >= {"decode_dma", "prefill_ks"}
    fake = tmp_path / "x.so"
    fake.write_bytes(b"\0junk__CLANG_OFFLOAD_BUNDLE__hipv4-amdgcn-amd-amdhsa--gfx942\0more")
    assert doctor._gfx_targets(str(fake)) == ["gfx942"]
    assert doctor.main(["--json"]) == (1 if rep["problems"] else 0)


@pytest.mark.gpu
def test_doctor_kernel_self_test_gpu():
    """The deployment check's GPU self-test (RMSNorm, decode-shape GEMM + SwiGLU, paged decode
    attention against fp32) passes on the box."""
    from nv_genai_amd.tools import doctor

    rep = doctor.collect(run_kernels=True)
    assert all(v["ok"] for v in rep["self_test"].values()), rep["self_test"]
    assert rep["gpus"] and rep["gpus"][0]["arch"].startswith("gfx950")
    assert not rep["problems"], rep["problems"]


def _smt_topology(root, ncpu=192, smt_offset=96, ccd_cores=12):
    """Fake cpu topology for _tree's node: CPU c and c + 96 are SMT siblings of one physical
    core; each CCD (L3 domain) holds 12 physical cores (24 logical CPUs), 4 CCDs per socket."""
    for c in range(ncpu):
        core = c % smt_offset
        sibs = f"{core},{core + smt_offset}"
        ccd = core // ccd_cores
        lo = ccd * ccd_cores
        l3 = f"{lo}-{lo + ccd_cores - 1},{lo + smt_offset}-{lo + smt_offset + ccd_cores - 1}"
        d = root / f"sys/devices/system/cpu/cpu{c}"
        (d / "topology").mkdir(parents=True)
        (d / "topology/thread_siblings_list").write_text(sibs + "\n")
        (d / "topology/core_id").write_text(f"{core % 48}\n")
        (d / "topology/physical_package_id").write_text(f"{core // 48}\n")
        (d / "cache/index3").mkdir(parents=True)
        (d / "cache/index3/shared_cpu_list").write_text(l3 + "\n")


def test_smt_siblings_and_l3_domains_stay_with_one_rank(tmp_path):
    """The round-5 plan sliced the node's cpulist contiguously, so on `0-47,96-143` rank 2 got
    96-119, the SMT siblings of rank 0's 0-23. Now every rank gets whole physical cores and,
    with one L3 domain (CCD) or more per rank, whole L3 domains."""
    root = _tree(tmp_path)
    _smt_topology(tmp_path)
    allowed = list(range(192))
    core_of = {c: c % 96 for c in range(192)}
    owner = {}
    for r in range(8):
        pl = affinity.plan(r, 8, root, env={}, allowed=allowed)
        assert len(pl.cpus) == 24 and pl.physical_cores == 12
        for c in pl.cpus:                          # both siblings of each core, no core shared
            assert owner.setdefault(core_of[c], r) == r
            assert (c + 96 if c < 96 else c - 96) in pl.cpus
        assert len(pl.l3_domains) == 1 and pl.whole_l3
        rec = pl.record()
        assert rec["physical_cores"] == 12 and rec["whole_l3"] and rec["l3_domains"] == pl.l3_domains
    # 8 ranks on one socket's 4 CCDs: whole cores (6 each), two ranks per CCD
    env = {"HIP_VISIBLE_DEVICES": "0,1,2,3"}
    owner = {}
    for r in range(8):
        pl = affinity.plan(r, 8, root, env=env, allowed=allowed)
        assert pl.numa_node == 0 and pl.physical_cores == 6 and len(pl.cpus) == 12
        assert len(pl.l3_domains) == 1 and not pl.whole_l3
        for c in pl.cpus:
            assert owner.setdefault(core_of[c], r) == r
    # 3 ranks over 4 CCDs: whole domains, balanced 2/1/1 by cores
    parts = affinity.split_cores(affinity.cpu_topology(affinity.parse_cpulist("0-47,96-143"), root), 3)
    assert [len(p) for p in parts] == [24, 12, 12]
    assert [len({c.l3 for c in p}) for p in parts] == [2, 1, 1]
    assert not ({c.l3 for c in parts[0]} & {c.l3 for c in parts[1]})


def test_visible_devices_hip_overrides_cuda(tmp_path):
    """HIP applies CUDA_VISIBLE_DEVICES only when HIP_VISIBLE_DEVICES is unset (not on top of
    it); ROCR_VISIBLE_DEVICES always filters first."""
    root = _tree(tmp_path)
    both = affinity.visible_gpus(root, env={"HIP_VISIBLE_DEVICES": "6,1", "CUDA_VISIBLE_DEVICES": "1"})
    assert [g.pci for g in both] == ["0000:65:00.0", "0000:15:00.0"]
    cuda = affinity.visible_gpus(root, env={"CUDA_VISIBLE_DEVICES": "1"})
    assert [g.pci for g in cuda] == ["0000:15:00.0"]
    rocr = affinity.visible_gpus(root, env={"ROCR_VISIBLE_DEVICES": "4,5,6", "HIP_VISIBLE_DEVICES": "2"})
    assert [g.pci for g in rocr] == ["0000:65:00.0"]
