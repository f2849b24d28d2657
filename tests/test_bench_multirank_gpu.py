"""The driver's multi-GPU bench path, rehearsed on the GPU box's single MI355X.

``python bench.py --gpus 2`` self-launches ``torch.distributed.run`` with two ranks. With fewer
GPUs than ranks, ``init_distributed`` maps the ranks round-robin onto the device and uses gloo
for the host-side groups (RCCL refuses two ranks of one communicator on one device), so every
GPU-side piece of the DP replica path runs: per-rank engines with hipGraphs, per-rank
indexes, the timed barriers and the max-over-ranks reduction. On an 8-GPU node the same
command runs one rank per GPU over RCCL.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(extra, shared=True, expect_ok=True):
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "1",
                        "--model", "llama-small", "--embed-model", "encoder-tiny", "--index-size", "20000",
                        "--concurrency", "8", "--max-tokens", "8", "--kv-cache-fraction", "0.02"] + extra
                       + (["--allow-shared-devices"] if shared else []),
                       cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    if not expect_ok:
        return r
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def _check_record(res, n):
    """The run record names every rank's device: on this box both ranks share one GPU."""
    dv = res["devices"]
    assert res["shared_devices"] is True and dv["backend"] == res["backend"]
    assert [r["rank"] for r in dv["ranks"]] == list(range(n))
    assert all(r["device"].startswith("cuda:") and r.get("pci_bus_id") is not None for r in dv["ranks"])
    assert dv["distinct_devices"] == 1


def test_bench_refuses_more_ranks_than_gpus():
    """Without --allow-shared-devices a 2-rank job on a 1-GPU box must not produce a record."""
    import torch

    if torch.cuda.device_count() != 1:
        pytest.skip("needs a box with exactly one GPU")
    r = _run([], shared=False, expect_ok=False)
    assert r.returncode != 0 and "refusing" in (r.stderr + r.stdout)
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_bench_two_dp_ranks_on_one_gpu():
    res = _run([])
    assert res["n_gpus"] == 2 and res["world_size"] == 2 and res["config"]["parallelism"] == "dp2"
    assert len(res["per_replica_qps"]) == 2 and res["value"] > 0
    assert res["config"]["global_batch"] == 16
    _check_record(res, 2)


def test_bench_tp2_replica_sharded_index_on_one_gpu():
    """One TP=2 replica with its index striped over both ranks: the follower replays the
    driver's steps and joins its sharded searches."""
    res = _run(["--tp", "2", "--sharded-index"])
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp1xtp2"
    assert res["value"] > 0
    _check_record(res, 2)
    # TP ranks record the custom all-reduce outcome (gloo host groups on shared devices: the
    # IPC all-reduce is built and self-tested, or reports why not)
    assert all("state" in r["custom_all_reduce"] for r in res["devices"]["ranks"])
