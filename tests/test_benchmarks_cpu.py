"""Benchmark harnesses run end to end on CPU with tiny models (their GPU numbers are in
BASELINE.md / profiles/)."""
import json
import os
import subprocess
import sys

import pytest


def test_multi_turn_benchmark_cpu(tmp_path):
    out = tmp_path / "mt.json"
    r = subprocess.run([sys.executable, "benchmarks/multi_turn.py", "--model", "llama-tiny", "--embed-model",
                        "encoder-tiny", "--index-size", "3000", "--sessions", "3", "--turns", "3",
                        "--warmup-sessions", "1", "--max-tokens", "5", "--out", str(out)],
                       capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=os.getcwd()))
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(out.read_text())
    # every turn wrote two memory entries; later turns retrieve history
    assert res["memory_entries"] == 2 * (1 * 3 + 3 * 3) and res["history_hits_per_turn"] > 0
    assert res["value"] > 0 and res["turns"] == 3


def test_http_rag_benchmark_cpu(tmp_path):
    """benchmarks/http_rag.py: chain-server process (developer_rag, in-process engines, synthetic
    collection, batched vector-store queries) driven over REST + SSE by the async load generator."""
    out = tmp_path / "http.json"
    r = subprocess.run([sys.executable, "benchmarks/http_rag.py", "--llm", "llama-tiny", "--embed", "encoder-tiny",
                        "--index-size", "3000", "--concurrency", "4", "--requests", "8", "--warmup", "2",
                        "--max-tokens", "6", "--device", "cpu", "--out", str(out)],
                       capture_output=True, text=True, timeout=400,
                       env=dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=os.getcwd(),
                                NGA_HTTP_BENCH_LOG=str(tmp_path / "server.log")))
    assert r.returncode == 0, (r.stderr[-3000:], (tmp_path / "server.log").read_text()[-3000:])
    res = json.loads(out.read_text())
    assert res["requests"] == 8 and res["value"] > 0 and res["p50_ttft_ms"] is not None
    # the server's own phase summaries and the engine counters over the timed window
    assert {"chain", "chain_wait", "prepare", "ttft"} <= set(res["server_p50_ms"]), res["server_p50_ms"]
    assert res["engine_window"]["steps"] > 0 and "wait" in res["engine_window"]["host_s"], res["engine_window"]
    pc = res["engine_window"]["prefix_cache"]
    assert pc["prompt_tokens_total"] > 0 and 0.0 <= pc["hit_share"] <= 1.0, pc


def test_http_rag_benchmark_split_topology_cpu(tmp_path):
    """--topology split: the reference's deployment — the chain server (developer_rag, index
    in-process) reaches the LLM and the query encoder through a separate model-server process
    over HTTP (OpenAI chat stream, base64 embeddings, whitened on the chain side); the engine
    counters come from the model server's /metrics."""
    out = tmp_path / "split.json"
    r = subprocess.run([sys.executable, "benchmarks/http_rag.py", "--llm", "llama-tiny", "--embed", "encoder-tiny",
                        "--topology", "split", "--index-size", "3000", "--concurrency", "4", "--requests", "8",
                        "--warmup", "2", "--max-tokens", "6", "--device", "cpu", "--out", str(out)],
                       capture_output=True, text=True, timeout=500,
                       env=dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=os.getcwd(),
                                NGA_HTTP_BENCH_LOG=str(tmp_path / "server.log")))
    assert r.returncode == 0, (r.stderr[-3000:], (tmp_path / "server.log").read_text()[-3000:])
    res = json.loads(out.read_text())
    assert res["topology"] == "split" and res["requests"] == 8 and res["value"] > 0
    assert res["sse_gap_ms"]["frames"] > 0
    ew = res["engine_window"]
    assert ew["steps"] > 0 and ew["prefix_cache"]["prompt_tokens_total"] > 0, ew
    assert "ttft" in res["model_server_p50_ms"], res["model_server_p50_ms"]   # the model server's own phases


def test_headline_bench_two_ranks_gloo(tmp_path):
    """bench.py under torch.distributed.run with 2 ranks (gloo on CPU, the driver's N>1 launch):
    exactly one JSON line, from rank 0, with the whole-job value over both replicas; rank 0's
    step timeline (--timeline-out) and its composition through scripts/steps_probe.py."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    tl = tmp_path / "timeline.json"
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr=127.0.0.1", f"--master-port={port}", "bench.py", "--gpus", "2",
                        "--steps", "1", "--warmup", "1", "--model", "llama-tiny", "--embed-model", "encoder-tiny",
                        "--index-size", "2000", "--concurrency", "3", "--max-tokens", "4",
                        "--timeline-out", str(tl)],
                       capture_output=True, text=True, timeout=400,
                       env=dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=os.getcwd()))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2"
    assert res["config"]["global_batch"] == 6 and res["steps"] == 1 and res["warmup"] == 1
    # value is the aggregate over ranks: 2 x 3 requests in the max-over-ranks time
    assert abs(res["value"] - 6 / (res["ms_per_step"] / 1000)) / res["value"] < 0.01
    for k in ("metric", "unit", "higher_is_better", "scaling", "vs_baseline", "dtype", "data"):
        assert k in res
    steps = json.loads(tl.read_text())
    assert steps and {"kind", "rows", "tokens", "decode_rows"} <= set(steps[0])
    assert sum(1 for st in steps if st["kind"] == "decode") > 0
    p = subprocess.run([sys.executable, "scripts/steps_probe.py", str(tl)], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    comp = json.loads(p.stdout)
    assert comp["decode"]["steps"] > 0


def test_headline_bench_self_launches_for_gpus_n():
    """``python bench.py --gpus 2`` (no torchrun around it): bench.py starts the 2-rank job
    itself as a child and relays rank 0's line, which reports both ranks."""
    env = dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=os.getcwd())
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "1",
                        "--model", "llama-tiny", "--embed-model", "encoder-tiny", "--index-size", "2000",
                        "--concurrency", "3", "--max-tokens", "4"],
                       capture_output=True, text=True, timeout=400, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["world_size"] == 2 and res["config"]["parallelism"] == "dp2"
    assert len(res["per_replica_qps"]) == 2 and res["config"]["global_batch"] == 6
    # the run record names each rank's device and the backend (CPU ranks here)
    assert res["shared_devices"] is False and res["devices"]["backend"] == "gloo"
    assert [r["rank"] for r in res["devices"]["ranks"]] == [0, 1]


def test_bench_refuses_shared_devices_without_flag(monkeypatch):
    """More ranks on the node than GPUs: refused unless --allow-shared-devices (then reported
    as shared); no GPUs at all (CPU rehearsal) or enough GPUs: allowed."""
    import bench
    import torch

    args = bench.parse(["--gpus", "8"])
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    with pytest.raises(SystemExit, match="refusing"):
        bench.check_devices(args, 8)
    assert bench.check_devices(bench.parse(["--gpus", "8", "--allow-shared-devices"]), 8) is True
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    assert bench.check_devices(args, 8) is False
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 0)
    assert bench.check_devices(args, 8) is False
    # multi-node: 16 ranks, 8 on this node with 8 GPUs
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    assert bench.check_devices(args, 16) is False
