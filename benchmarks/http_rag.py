"""End-to-end RAG QPS through the REST API: the headline workload of bench.py, but every request
is a real ``POST /generate`` (``use_knowledge_base: true``, SSE stream) to the chain server.

The chain server (``developer_rag`` example, uvicorn) runs in its own process with in-process
engines on the GPU. It uses ``APP_LLM_MODELENGINE=local`` and
``APP_EMBEDDINGS_MODELENGINE=local``, and a synthetic 1M-chunk collection
(``APP_INDEX_SYNTHETICDOCS``). Concurrent requests' searches are coalesced by the vector store's
query batcher on its own HIP stream. Generation goes through the continuous-batching engine.

The load generator is a separate CPU-only asyncio process. It runs a closed loop: each of
``--concurrency`` clients posts a generated question, reads the SSE stream to ``[DONE]`` and posts
the next. Clients start staggered over ``--ramp-s`` (bench.py ramps its clients in the same
way), so arrivals are spread in time rather than synchronized into waves that all prefill at
once. Once ``--warmup`` requests have completed, the next ``--requests`` completions are
timed, with every client still busy (no drain inside the window, as in bench.py). The script
prints one JSON line with QPS and the p50/p95 latency and TTFT of the timed requests.

``--topology split`` runs the reference's deployed shape instead
(``deploy/compose/docker-compose-nim-ms.yaml:1-84``, ``common/utils.py:265-316``): the LLM and
the embedding encoder are served by ``serving/model_server.py`` (OpenAI / NIM API) in a second
process on the same GPU, and the chain server reaches them over HTTP
(``APP_LLM_MODELENGINE=nim``, ``APP_EMBEDDINGS_MODELENGINE=nim``); the index stays in the chain
server. ``--stream-interval`` sets ``NGA_STREAM_INTERVAL`` in the serving processes (1, the
default: one SSE frame per generated token, as the reference streams). The JSON reports the
gaps between a stream's SSE frames (p50 / p99 over the timed requests).

Each request follows the reference's path, not bench.py's. The chain server forwards only
temperature, top_p and max_tokens (utils.py:271-286 quirk), so generation may stop early at an
EOS token. Output tokens are therefore counted from the streamed text and reported.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _server_quantiles(text: str, prefix: str = "chain_server_") -> dict:
    """p50 (ms) of a server's own request-phase summaries (whole run, warmup included). Chain
    server: chain_wait = request arrival -> retrieval + prompt queued on the engine (worker-thread
    queueing included), chain = that work alone, ttft = arrival -> first token. Model server
    (split topology): ttft / request = its own receipt of the chat request -> first token / end,
    embed = one /v1/embeddings call."""
    out = {}
    for line in text.splitlines():
        if line.startswith(prefix) and 'quantile="0.5"' in line:
            name = line.split("{")[0][len(prefix):]
            if name == "retrieval_batch_size":
                out[name] = float(line.rsplit(" ", 1)[1])
            elif name.endswith("_seconds"):
                try:
                    out[name[:-len("_seconds")]] = round(1e3 * float(line.rsplit(" ", 1)[1]), 2)
                except ValueError:
                    pass
    return out


def _gauges(text: str, prefix: str = "chain_server_") -> dict:
    out = {}
    for line in text.splitlines():
        if line.startswith(prefix) and "{" not in line:
            k, _, v = line.partition(" ")
            try:
                out[k[len(prefix):]] = float(v)
            except ValueError:
                pass
    return out


def _engine_window(m0, m1) -> dict:
    """Engine counters over the timed window (same fields as bench.py's ``host_s``): steps by
    kind and host seconds per phase; ``wait`` is the engine thread blocked on the GPU."""
    if not m0 or not m1:
        return {}
    d = {k: m1[k] - m0.get(k, 0.0) for k in m1 if k in m0}
    steps = d.get("steps", 0.0)
    out = {"steps": int(steps), "decode_steps": int(d.get("decode_steps", 0)), "mixed_steps": int(d.get("mixed_steps", 0)),
           "host_s": {k[5:-2]: round(d.get(k, 0.0), 3) for k in ("host_sched_s", "host_launch_s", "host_between_s",
                                                                 "host_wait_s", "host_finalize_s")}}
    if steps:
        out["host_ms_per_step"] = {k: round(1e3 * v / steps, 3) for k, v in out["host_s"].items()}
    if "prefix_hit_blocks" in d and "prefill_tokens" in d:
        # prompt tokens served from the prefix cache (64-token blocks) vs computed in prefill:
        # the same share bench.py reports, so the two topologies are comparable
        hit = 64 * d["prefix_hit_blocks"]
        tot = hit + d["prefill_tokens"]
        out["prefix_cache"] = {"hit_tokens": int(hit), "prompt_tokens_total": int(tot),
                               "hit_share": round(hit / tot, 4) if tot else 0.0}
    return out


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--llm", default="llama3-8b")
    ap.add_argument("--embed", default="arctic-embed-l")
    ap.add_argument("--index-size", type=int, default=1_000_000)
    ap.add_argument("--concurrency", type=int, default=256)
    ap.add_argument("--requests", type=int, default=2048)
    ap.add_argument("--warmup", type=int, default=256)
    ap.add_argument("--max-tokens", type=int, default=256)
    ap.add_argument("--ramp-s", type=float, default=6.0,
                    help="client k starts k/concurrency * ramp_s after the first (0: all at once)")
    ap.add_argument("--example", default="developer_rag")
    ap.add_argument("--device", default="", help="engine device for the server ('' = cuda if available)")
    ap.add_argument("--startup-timeout", type=float, default=600.0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--topology", choices=("inprocess", "split"), default="inprocess",
                    help="split: LLM + encoder in a model-server process, reached over HTTP")
    ap.add_argument("--stream-interval", type=int, default=1,
                    help="NGA_STREAM_INTERVAL of the serving processes (1: a frame per token)")
    return ap.parse_args(argv)


async def _one(client, url, question, max_tokens, gaps=None):
    t0 = time.perf_counter()
    ttft = None
    chars = 0
    last = None
    body = {"messages": [{"role": "user", "content": question}], "use_knowledge_base": True,
            "temperature": 0.2, "top_p": 0.7, "max_tokens": max_tokens}
    async with client.stream("POST", url, json=body) as r:
        if r.status_code != 200:
            raise RuntimeError(f"/generate returned {r.status_code}")
        async for line in r.aiter_lines():
            if not line.startswith("data: "):
                continue
            frame = json.loads(line[6:])
            ch = frame["choices"][0]
            text = ch["message"]["content"]
            now = time.perf_counter()
            if text and ttft is None:
                ttft = now - t0
            if text:
                if last is not None and gaps is not None:
                    gaps.append(now - last)
                last = now
            chars += len(text)
            if ch.get("finish_reason") == "[DONE]":
                break
    return time.perf_counter() - t0, ttft, chars


async def _load(url, args, questions):
    """Closed loop without a drain in the timed window (like bench.py): every client keeps a
    request in flight; completions are counted from the moment ``--warmup`` requests have
    completed until ``--requests`` more have, while every client is still busy."""
    import httpx

    metrics_url = args.engine_metrics_url or url.rsplit("/", 1)[0] + "/metrics"
    prefix = args.engine_metrics_prefix
    limits = httpx.Limits(max_connections=args.concurrency + 8, max_keepalive_connections=args.concurrency + 8)
    results = []
    state = {"done": 0, "t_start": None, "stop": False, "issued": 0}

    async def client_loop(client, k):
        # staggered start (bench.py's ramp): client k joins k/concurrency of the way through
        # one request's lifetime, so completions and re-arrivals spread evenly over time
        # instead of all clients prefilling together in synchronized waves
        await asyncio.sleep(k * args.ramp_s / max(1, args.concurrency))
        while not state["stop"]:
            i = state["issued"]
            state["issued"] += 1
            g = []
            lat, ttft, chars = await _one(client, url, questions[i % len(questions)], args.max_tokens, g)
            now = time.perf_counter()
            state["done"] += 1
            if state["done"] == args.warmup:
                state["t_start"] = now
                state["m0"] = _gauges((await client.get(metrics_url)).text, prefix)
            elif state["t_start"] is not None and not state["stop"]:
                results.append((lat, ttft, chars, now))
                state.setdefault("gaps", []).extend(g)
                if len(results) >= args.requests:
                    state["stop"] = True
                    state["m1"] = _gauges((await client.get(metrics_url)).text, prefix)

    async with httpx.AsyncClient(timeout=httpx.Timeout(600.0), limits=limits) as client:
        await asyncio.gather(*(client_loop(client, k) for k in range(args.concurrency)))
    return results, state["t_start"], _engine_window(state.get("m0"), state.get("m1")), state.get("gaps", [])


def _wait_up(proc, url, log_path, timeout):
    import httpx

    t0 = time.time()
    while True:
        if proc.poll() is not None:
            raise RuntimeError(f"server exited ({proc.returncode}); see {log_path}")
        try:
            if httpx.get(url, timeout=5).status_code == 200:
                return
        except Exception:  # noqa: BLE001 - not up yet
            pass
        if time.time() - t0 > timeout:
            raise RuntimeError(f"server at {url} did not come up; see {log_path}")
        time.sleep(1.0)


def _embed_dim(preset: str) -> int:
    from nv_genai_amd.models.config import encoder_config

    return encoder_config(preset).hidden


def _pct(xs, q):
    if not xs:
        return None
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))]


def main(argv=None):
    args = parse(argv)
    from nv_genai_amd.utils.synthetic import TextGen

    port = _free_port()
    log_dir = os.path.dirname(os.environ.get("NGA_HTTP_BENCH_LOG", os.path.join(ROOT, "gpurun_out", "x")))
    os.makedirs(log_dir, exist_ok=True)
    common = dict(os.environ, PYTHONPATH=ROOT, LOGLEVEL=os.environ.get("LOGLEVEL", "WARNING"),
                  NGA_STREAM_INTERVAL=str(args.stream_interval))
    env = dict(common, EXAMPLE_NAME=args.example, APP_INDEX_SYNTHETICDOCS=str(args.index_size),
               APP_ENGINE_MAXNUMSEQS=str(max(args.concurrency, 1)), APP_ENGINE_DEVICE=args.device)
    procs = []
    args.engine_metrics_url, args.engine_metrics_prefix = None, "chain_server_"
    if args.topology == "split":
        mport = _free_port()
        mlog_path = os.path.join(log_dir, "http_rag_model_server.log")
        cmd = [sys.executable, "-m", "nv_genai_amd.serving.model_server", "--llm", args.llm, "--embed", args.embed,
               "--host", "127.0.0.1", "--port", str(mport), "--max-num-seqs", str(max(args.concurrency, 1))]
        if args.device:
            cmd += ["--device", args.device]
        procs.append(subprocess.Popen(cmd, env=dict(common, LOGLEVEL="warning"), stdout=open(mlog_path, "w"),
                                      stderr=subprocess.STDOUT))
        _wait_up(procs[-1], f"http://127.0.0.1:{mport}/v1/health/ready", mlog_path, args.startup_timeout)
        murl = f"http://127.0.0.1:{mport}/v1"
        env.update(APP_LLM_MODELENGINE="nim", APP_LLM_SERVERURL=murl, APP_LLM_MODELNAME=args.llm,
                   APP_EMBEDDINGS_MODELENGINE="nim", APP_EMBEDDINGS_SERVERURL=murl,
                   APP_EMBEDDINGS_MODELNAME=args.embed, APP_EMBEDDINGS_DIMENSIONS=str(_embed_dim(args.embed)))
        args.engine_metrics_url = f"http://127.0.0.1:{mport}/metrics"
        args.engine_metrics_prefix = "model_server_"
    else:
        env.update(APP_LLM_MODELENGINE="local", APP_EMBEDDINGS_MODELENGINE="local",
                   APP_ENGINE_LLMPRESET=args.llm, APP_ENGINE_EMBEDPRESET=args.embed)
    log_path = os.environ.get("NGA_HTTP_BENCH_LOG", os.path.join(log_dir, "http_rag_server.log"))
    log = open(log_path, "w")
    procs.append(subprocess.Popen([sys.executable, "-m", "uvicorn", "nv_genai_amd.chain_server.server:app",
                                   "--host", "127.0.0.1", "--port", str(port), "--log-level", "warning"],
                                  env=env, stdout=log, stderr=subprocess.STDOUT))
    server = procs[-1]
    try:
        import httpx

        base = f"http://127.0.0.1:{port}"
        t0 = time.time()
        _wait_up(server, base + "/health", log_path, args.startup_timeout)
        # first search builds the engines and fills the synthetic collection
        httpx.post(base + "/search", json={"query": "warm up", "top_k": 4}, timeout=args.startup_timeout)
        setup_s = time.time() - t0
        print(f"[http_rag] servers up ({setup_s:.0f} s), topology {args.topology}", file=sys.stderr, flush=True)
        gen = TextGen(seed=100)
        questions = [gen.question() for _ in range(4096)]
        results, t_start, engine_window, gaps = asyncio.run(_load(base + "/generate", args, questions))
        server_side = _server_quantiles(httpx.get(base + "/metrics", timeout=30).text)
        model_side = (_server_quantiles(httpx.get(args.engine_metrics_url, timeout=30).text, "model_server_")
                      if args.topology == "split" else None)
        t_end = max(r[3] for r in results)
        elapsed = t_end - t_start
        lat = sorted(r[0] for r in results)
        ttft = sorted(r[1] for r in results if r[1] is not None)
        res = {"metric": "end-to-end RAG QPS + p50 latency through the chain-server REST API (POST /generate, SSE)",
               "value": round(len(results) / elapsed, 4), "unit": "requests/s", "n_gpus": 1,
               "requests": len(results), "concurrency": args.concurrency, "elapsed_s": round(elapsed, 3),
               "ramp_s": args.ramp_s, "topology": args.topology, "stream_interval": args.stream_interval,
               "p50_latency_ms": round(1e3 * statistics.median(lat), 1),
               "p95_latency_ms": round(1e3 * lat[min(len(lat) - 1, int(0.95 * len(lat)))], 1),
               "p50_ttft_ms": round(1e3 * statistics.median(ttft), 1) if ttft else None,
               # time between consecutive text frames of one stream (per-token streaming: ~one
               # engine step; an interval of N steps: ~N steps)
               "sse_gap_ms": {"p50": round(1e3 * _pct(gaps, 0.5), 2) if gaps else None,
                              "p99": round(1e3 * _pct(gaps, 0.99), 2) if gaps else None,
                              "frames": len(gaps) + len(results)},
               "mean_output_chars": round(sum(r[2] for r in results) / len(results), 1),
               "config": {"model": f"{args.llm} + {args.embed}", "index_size": args.index_size,
                          "example": args.example, "max_tokens": args.max_tokens},
               "dtype": "bf16", "data": "synthetic: random-init weights, 1M random unit-vector index, generated questions",
               "setup_s": round(setup_s, 1), "server_p50_ms": server_side,
               **({"model_server_p50_ms": model_side} if model_side is not None else {}),
               "engine_window": engine_window}
        line = json.dumps(res)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")
    finally:
        for p in reversed(procs):
            p.terminate()
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()


if __name__ == "__main__":
    main()
