#!/usr/bin/env python3
"""Headline benchmark: end-to-end RAG QPS + p50 latency, Llama-3-8B + arctic-embed-l,
1M-doc index (BASELINE.json ``metric``).

One rank per GPU (``torch.distributed.run``; RCCL for the barrier / max-reduce of the
timing). Each rank is a full serving replica (data parallel, SURVEY.md §2.E "DP (data /
replica)", CC9): Llama-3-8B engine + arctic-embed-l encoder + a 1M x 1024 in-HBM flat index
(2 GB, replicated: cheaper than any per-query collective at this size).

Every request is served end to end inside the timed region: query embedding (encoder
forward), top-4 cosine search over the 1M-vector index, 1500-token context cap, prompt
assembly with the reference ``rag_template`` + Llama-3 chat template, continuous-batched
prefill + decode of ``--max-tokens`` tokens (EOS ignored so every request does the same
work), streaming detokenisation.

Load model (``--mode``):
* ``closed`` (default): ``--concurrency`` closed-loop clients per GPU — each client sends
  its next question as soon as its previous answer completes (the usual serving-benchmark
  load). Clients ramp up one request lifetime apart so the run reaches steady state; a
  *step* is ``--concurrency`` completed requests, so ``--steps K`` times K·C completions
  after ``--warmup W``·C warm-up completions. Steady state is what mixed prefill/decode
  batching is built for: each engine step decodes every running request and prefills the
  newly arrived ones in the same GEMMs.
* ``wave``: a step is one synchronized wave of C requests submitted together.

Weights are random-init of the real architectures; the corpus is synthetic (index vectors
are random unit vectors standing in for arctic-embed-l passage embeddings; chunk texts are
generated prose of ~500 tokens). ``value`` is the whole-job QPS (all ranks).

Launch: ``python bench.py --gpus N`` with N > 1 and no ``WORLD_SIZE`` in the environment starts
``torch.distributed.run --nproc-per-node N`` on this same command line as a child process
(before anything touches the GPU) and exits with its status; under torchrun the job checks
``WORLD_SIZE == --gpus``.

Model parallelism (``--tp T``, SURVEY.md §2.E TP; the reference's ``tensor_para_size`` /
``enable_custom_all_reduce``, experimental/fm-asr-streaming-rag/nim/configs/mistral-7b.yaml:32-36,
and NIM's ``count: ${INFERENCE_GPU_COUNT:-all}``, deploy/compose/docker-compose-nim-ms.yaml:20):
the N ranks form N / T replicas of T ranks each; every replica's driver (tp rank 0) serves the
RAG clients, its followers replay the driver's steps over RCCL (TP all-reduces on xGMI). With
``--sharded-index`` the replica's index is striped over its T ranks and each search is a
broadcast + per-shard MFMA top-k + all-gather merge (CC7/CC8) on the replica's step channel.

``--workload agent`` runs the query-decomposition agent (BASELINE.json configs[3]: Llama-3-70B
TP=N + a 10M-vector index sharded over the N ranks; ``benchmarks/agent_tp.py``) and reports
agent queries/s in the same JSON shape.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

import torch


REF_EQUIV_QPS_PER_GPU = 4.40   # profiles/r1_refeq/ref_eq.json
SEARCH_CMD = -3    # replica step-channel command: sharded search (followers join the collectives)
BARRIER_CMD = -4   # replica step-channel command: followers join a world barrier


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--concurrency", type=int, default=256, help="requests per rank per step")
    ap.add_argument("--max-tokens", type=int, default=256)
    ap.add_argument("--index-size", type=int, default=1_000_000)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--embed-model", default="arctic-embed-l")
    ap.add_argument("--top-k", type=int, default=4)
    ap.add_argument("--max-batched-tokens", type=int, default=32768)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--profile-dir", default=None, help="write a torch.profiler trace here")
    ap.add_argument("--out", default=None, help="also write the JSON line to this file")
    ap.add_argument("--timeline-out", default=None,
                    help="write the engine's last 4,096 scheduler steps (kind, rows, tokens, decode rows) here")
    ap.add_argument("--no-step-timing", dest="step_timing", action="store_false",
                    help="skip the GPU events around every engine step (in-step time vs idle between "
                         "steps, reported as gpu_step_timing; on by default, two event records per step)")
    ap.add_argument("--step-timing", dest="step_timing", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--mode", choices=("closed", "wave"), default="closed")
    ap.add_argument("--fp8", action="store_true",
                    help="W8A8 FP8 projections (not the headline: that is measured in bf16)")
    ap.add_argument("--kv-fp8", action="store_true",
                    help="FP8 e4m3fn KV cache (not the headline: that is measured in bf16)")
    ap.add_argument("--mixed-prefill-tokens", type=int, default=4096,
                    help="prefill tokens per mixed step (sweep: profiles/r2_mixed_sweep)")
    ap.add_argument("--mixed-min-tokens", type=int, default=0,
                    help="accumulate this many prompt tokens before forming a mixed step")
    ap.add_argument("--mixed-max-wait", type=int, default=4)
    ap.add_argument("--retrieval-batch", type=int, default=8,
                    help="queries per embedding+search launch (dynamic batching, like the reference's Triton embedder)")
    ap.add_argument("--no-quiet-gc", action="store_true",
                    help="keep CPython's default GC (multi-ms host pauses stall the GPU)")
    ap.add_argument("--retrieval-delay-ms", type=float, default=50.0,
                    help="max time a query waits for its retrieval batch to fill (Triton max_queue_delay)")
    ap.add_argument("--tp", type=int, default=1,
                    help="tensor-parallel ranks per replica (N / tp replicas)")
    ap.add_argument("--sharded-index", action="store_true",
                    help="stripe each replica's index over its tp ranks (broadcast + all-gather merge)")
    ap.add_argument("--workload", choices=("rag", "agent"), default="rag",
                    help="agent: query-decomposition agent, one TP=N replica + N-way sharded index")
    ap.add_argument("--kv-cache-fraction", type=float, default=None)
    ap.add_argument("--no-step-graphs", action="store_true",
                    help="prefill / mixed steps eagerly (A/B of the step hipGraphs)")
    ap.add_argument("--graph-token-step", type=int, default=None,
                    help="token-count bucket of the prefill / mixed step graphs (engine default)")
    ap.add_argument("--no-prefix-cache", dest="prefix_cache", action="store_false",
                    help="turn the engine's prefix cache off (the A/B of the hit share the JSON reports)")
    ap.add_argument("--allow-shared-devices", action="store_true",
                    help="let more ranks than GPUs share devices (a multi-rank rehearsal on a small box: "
                         "gloo host groups, not a scaling record)")
    return ap.parse_args(argv)


def check_devices(args, world: int) -> bool:
    """Refuse a GPU job with more ranks on this node than GPUs unless --allow-shared-devices:
    such a run shares devices and swaps RCCL for gloo, so its record must not pass for an
    N-GPU scaling point. Counting devices does not initialise the GPU on this image. Returns
    whether devices are shared."""
    if world <= 1:
        return False
    ngpu = torch.cuda.device_count()
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    if ngpu == 0 or local_world <= ngpu:
        return False
    if not args.allow_shared_devices:
        raise SystemExit(f"bench.py: {local_world} ranks on this node but only {ngpu} GPU(s); refusing to "
                         "record a multi-GPU result on shared devices (pass --allow-shared-devices to rehearse)")
    return True


def rank_devices(pctx) -> dict:
    """Run record of where the job ran: every rank's device index, name and PCI bus id, the
    backend and the RCCL version, and (tensor parallel) the custom all-reduce outcome."""
    from nv_genai_amd.parallel import dist as pd

    me = {"rank": pctx.rank, "local_rank": pctx.local_rank, "device": str(pctx.device)}
    if pd.PLACEMENT is not None:   # CPU / NUMA binding made before the GPU was touched
        me.update(pd.PLACEMENT.record())
    if pctx.device.type == "cuda":
        pr = torch.cuda.get_device_properties(pctx.device)
        me.update(name=pr.name, pci_bus_id=getattr(pr, "pci_bus_id", None),
                  pci_device_id=getattr(pr, "pci_device_id", None), pci_domain_id=getattr(pr, "pci_domain_id", None))
    if pctx.tp_size > 1:
        from nv_genai_amd.parallel.custom_ar import status

        me["custom_all_reduce"] = status()
    ranks = pd.all_gather_objects(me)
    rec = {"ranks": ranks, "backend": pctx.backend,
           "distinct_devices": len({(r.get("pci_domain_id"), r.get("pci_bus_id"), r.get("pci_device_id"), r["device"])
                                    for r in ranks})}
    if pctx.backend == "nccl":
        try:
            v = torch.cuda.nccl.version()
            rec["rccl_version"] = ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
        except Exception as e:  # noqa: BLE001
            rec["rccl_version"] = f"unavailable ({e!r})"[:80]
    return rec


def progress(msg: str, on: bool = True) -> None:
    """One progress line on stderr (the JSON result alone goes to stdout)."""
    if on:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(args) -> None:
    """``--gpus N > 1`` outside torchrun: run this command line under
    ``torch.distributed.run --nproc-per-node N`` as a child (no exec: nothing here has touched
    the GPU, but the child owns the devices) and exit with its status. Rank 0 prints the JSON
    line on the inherited stdout."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)]
    cmd += sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    root = os.path.dirname(os.path.abspath(__file__))
    env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    sys.stdout.flush()
    rc = subprocess.call(cmd, env=env)
    sys.exit(rc)


def host_step_summary(llm) -> dict:
    """Median / p90 / max (ms) of each host segment of the timed pipelined steps, and the
    same for the steps whose wait for the previous step was < 1 ms (the GPU had already
    finished it: a pipeline bubble unless the step was already queued)."""
    st = list(llm._host_steps)
    if not st:
        return {}
    names = ("outside", "pre_sched", "sched", "launch", "between", "wait", "finalize")
    seg = []
    prev_exit = None
    for e in st:
        enter, sch, h0, h1, h2, h3, ex = e
        seg.append((enter - prev_exit if prev_exit is not None else 0.0, sch - enter, h0 - sch,
                    h1 - h0, h2 - h1, h3 - h2, ex - h3))
        prev_exit = ex

    def stats(rows):
        out = {}
        for i, n in enumerate(names):
            v = sorted(r[i] for r in rows)
            if v:
                out[n] = [round(1e3 * v[len(v) // 2], 2), round(1e3 * v[int(0.9 * (len(v) - 1))], 2),
                          round(1e3 * v[-1], 2)]
        return out

    short = [r for r in seg if r[5] < 1e-3]
    return {"steps": len(seg), "all": stats(seg), "short_wait_steps": len(short),
            "short_wait": stats(short)}


class ReplicaSearch:
    """A replica-sharded index seen from the replica's driver: each search first announces
    itself on the step channel so the followers join its broadcast / all-gather."""

    def __init__(self, llm, index, src: int):
        self.llm, self.index, self.src = llm, index, src
        self.dim = index.dim

    def search(self, q, k):
        payload = self.index.query_payload(q)
        if payload.nbytes <= self.llm.command_payload_capacity():
            # the query block travels in the command itself: one collective per search
            self.llm.broadcast_command(SEARCH_CMD, int(q.shape[0]), payload)
            return self.index.search(q, k, have_queries=True)
        self.llm.broadcast_command(SEARCH_CMD, int(q.shape[0]))
        return self.index.search(q, k, src=self.src)


def run_agent(args, world: int, shared: bool = False) -> None:
    """``--workload agent``: benchmarks/agent_tp.py (one TP=world replica, world-way sharded
    index), ``--steps`` x ``--concurrency`` timed agent queries, reported in bench.py's shape."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from benchmarks import agent_tp

    model = args.model if args.model != "llama3-8b" else "llama3-70b"
    index_size = args.index_size if args.index_size != 1_000_000 else 10_000_000
    conc = args.concurrency if args.concurrency != 256 else 32
    argv = ["--model", model, "--embed-model", args.embed_model, "--index-size", str(index_size),
            "--queries", str(max(1, args.steps * conc)), "--warmup", str(args.warmup * conc),
            "--concurrency", str(conc), "--answer-tokens", str(args.max_tokens),
            "--top-k", str(args.top_k)]
    if args.no_graphs:
        argv.append("--no-graphs")
    if args.fp8:
        argv.append("--fp8")
    if args.kv_cache_fraction is not None:
        argv += ["--kv-cache-fraction", str(args.kv_cache_fraction)]
    res = agent_tp.main(argv, emit=False, record_devices=rank_devices if world > 1 else None)
    if res is None:          # follower rank
        return
    ms = 1000.0 * res["elapsed_s"] / max(1, args.steps)
    line = {
        "metric": f"query-decomposition agent QPS + p50 latency, {model} TP={world} + "
                  f"{index_size}-vector index sharded over {world} ranks",
        "value": res["value"], "unit": "agent queries/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 2), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": res["dtype"],
        "data": res["data"] + " (scripted agent decisions: the weights are random)",
        "config": {"model": f"{model} + {args.embed_model}", "global_batch": conc,
                   "seq_len": int(res["mean_prompt_tokens"]) + args.max_tokens,
                   "parallelism": f"tp{world}", "index_size": index_size, "sharded_index": world > 1,
                   "workload": "agent"},
        **{k: res[k] for k in ("p50_latency_ms", "p95_latency_ms", "llm_calls_per_s", "searches_per_s",
                               "mean_prompt_tokens", "output_tokens_per_s", "setup_s")},
        "world_size": world, "backend": res.get("backend"), "shared_devices": shared,
        **({"search": res["search"]} if res.get("search") else {}),
        **({"devices": res["devices"]} if res.get("devices") else {}),
    }
    s = json.dumps(line)
    print(s, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(s + "\n")


def main(argv=None):
    args = parse(argv)
    self_launch(args)
    if os.environ.get("NGA_STACK_DUMP_S"):
        # hang diagnosis: every rank dumps all its threads' Python stacks to stderr periodically
        import faulthandler

        faulthandler.dump_traceback_later(float(os.environ["NGA_STACK_DUMP_S"]), repeat=True)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env} ranks were launched")
    if world_env > 1:
        from nv_genai_amd.parallel.dist import bind_numa

        bind_numa()   # each rank on its GPU's NUMA node's cores, before any HIP call
    shared = check_devices(args, world_env)
    if args.workload == "agent":
        run_agent(args, world_env, shared)
        return
    if world_env > 1:
        # one rank per GPU on a shared host: give each rank's tokenizer thread pool (Rust
        # rayon, sized to every core by default) its share of the cores, before first use
        ncpu = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
        os.environ.setdefault("RAYON_NUM_THREADS", str(max(1, ncpu // world_env)))
    from nv_genai_amd.engine.embed_engine import EmbeddingEngine
    from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine, SamplingParams
    from nv_genai_amd.index.docstore import SyntheticDocStore
    from nv_genai_amd.index.flat import FlatIndex
    from nv_genai_amd.parallel import dist as pd
    from nv_genai_amd.rag.pipeline import RAGPipeline
    from nv_genai_amd.utils.synthetic import TextGen

    tp = max(1, args.tp)
    if world_env % tp:
        raise SystemExit(f"bench.py: --tp {tp} does not divide {world_env} ranks")
    pctx = pd.init_distributed(tp_size=tp)
    world, rank = pctx.world_size, pctx.rank
    assert world == args.gpus, (world, args.gpus)
    replicas = world // tp
    devices = None   # per-rank run record, collected after the timed region (rank_devices)
    dev = str(pctx.device)
    gpu = pctx.device.type == "cuda"
    if world > 1:
        # one rank per GPU on a shared host: split the intra-op CPU pool instead of letting
        # every rank spin up a full-width one (the host work is a single Python loop per rank)
        ncpu = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
        torch.set_num_threads(max(1, min(torch.get_num_threads(), (ncpu or 1) // world)))
    t_setup = time.time()
    R = args.concurrency
    # graphs for the padded decode batch sizes this run can see
    sizes = tuple(b for b in (1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 160, 192, 224, 256) if b <= R) or (1,)
    if sizes[-1] < R:
        sizes = sizes + (R,)
    kv_frac = args.kv_cache_fraction if args.kv_cache_fraction is not None else 0.3
    ecfg = EngineConfig(model=args.model, max_num_seqs=max(R, 1), max_batched_tokens=args.max_batched_tokens,
                        max_model_len=8192, use_graphs=gpu and not args.no_graphs,
                        graph_batch_sizes=sizes, seed=pctx.dp_rank, kv_cache_fraction=kv_frac,
                        kv_cache_blocks=None if gpu else 512,
                        mixed_prefill_tokens=args.mixed_prefill_tokens,
                        mixed_min_tokens=args.mixed_min_tokens, mixed_max_wait=args.mixed_max_wait,
                        fp8=args.fp8, kv_cache_dtype="fp8" if args.kv_fp8 else "auto",
                        mixed_graphs=not args.no_step_graphs, enable_prefix_caching=args.prefix_cache,
                        **({"graph_token_step": args.graph_token_step} if args.graph_token_step else {}))
    llm = LLMEngine(ecfg, device=dev, pctx=pctx)
    progress(f"engine up ({time.time() - t_setup:.0f} s)", llm.is_driver)
    from nv_genai_amd.models.config import encoder_config

    dim = encoder_config(args.embed_model).hidden
    sharded = args.sharded_index and tp > 1
    if sharded:
        from nv_genai_amd.index.sharded import ShardedIndex

        shard = ShardedIndex(dim, "cosine", dev, pctx=pctx, group=pctx.mp_group,
                             capacity=args.index_size // tp + 1)
        shard.add_random(args.index_size, seed=1234)
    if not llm.is_driver:
        # follower of a TP replica: replay the driver's steps; join its sharded searches and
        # the timing barriers; leave when the driver stops the replica
        hooks = {BARRIER_CMD: lambda n: (torch.cuda.synchronize() if gpu else None, pd.barrier())}
        if sharded:
            def search_hook(n, payload=None):
                if payload is not None:   # the driver's query block, from the command: side stream
                    return shard.search_side(payload, n, args.top_k, wait=False)
                return shard.search(torch.zeros(n, dim, device=shard.comm_dev), args.top_k, src=pctx.mp_src)
            hooks[SEARCH_CMD] = search_hook
        llm.run_follower(hooks=hooks)
        pd.all_reduce_max(0.0)
        pd.all_gather_objects(None)
        rank_devices(pctx)
        pd.destroy()
        return
    emb = EmbeddingEngine(args.embed_model, device=dev, seed=pctx.dp_rank)
    if sharded:
        index = ReplicaSearch(llm, shard, pctx.mp_src)
    else:
        index = FlatIndex(emb.dim, "cosine", dev, capacity=args.index_size)
        index.add_random(args.index_size, seed=1234)
    progress(f"index up ({time.time() - t_setup:.0f} s)")
    docs = SyntheticDocStore(args.index_size)
    rag = RAGPipeline(llm, emb, index, docs, top_k=args.top_k)
    gen = TextGen(seed=100 + pctx.dp_rank)

    def world_barrier():
        """Every rank, followers included (through the replica's step channel)."""
        llm.broadcast_command(BARRIER_CMD)
        if gpu:
            torch.cuda.synchronize()
        pd.barrier()
    # random-init encoder outputs are highly anisotropic (every query would retrieve the same
    # few passages and share KV through the prefix cache): PCA-whiten them so concurrent
    # queries retrieve different passages, as with a trained embedding model
    cal = TextGen(seed=999)
    emb.calibrate_whitening([cal.question() for _ in range(4096)])
    params = SamplingParams(temperature=0.2, top_p=0.7, max_tokens=args.max_tokens, ignore_eos=True)
    if gpu:
        torch.cuda.synchronize()
    setup_s = time.time() - t_setup

    def one_step():
        qs = [gen.question() for _ in range(R)]
        return rag.run(qs, params)

    active = {}                     # request id -> RAGResult of the closed-loop clients
    hostprof = {"poll": [], "submit": [], "work": []}
    ramp = max(1, -(-R // max(1, args.max_tokens)))  # new clients per engine step while ramping

    pending = []                    # retrievals in flight on the retrieval stream
    queued = []                     # (question, arrival time) waiting for a retrieval batch
    clients = [0]                   # clients with a question in the system (retrieving or generating)

    def closed_loop(n_done: int, ramping: bool, st_name: str = "step"):
        """Serve until ``n_done`` requests complete; a completed client re-submits at once.
        The client/retrieval host work (prompts for finished retrievals, the next retrieval
        batch on the retrieval stream) runs inside ``llm.step`` between launching the next
        engine step and waiting for the previous one, i.e. while the GPU is busy."""
        out = []
        st = {"ramping": ramping}

        def host_work(block: bool = False):
            hw0 = time.perf_counter()
            for res in rag.poll(pending, block=block):
                active[res.request.id] = res
            hw1 = time.perf_counter()
            need = R - clients[0]
            if st["ramping"]:
                need = min(need, ramp)
            if need > 0:
                now = time.perf_counter()
                queued.extend((gen.question(), now) for _ in range(need))
                clients[0] += need
            if queued and (len(queued) >= args.retrieval_batch or not llm.has_work()
                           or time.perf_counter() - queued[0][1] >= args.retrieval_delay_ms / 1e3):
                hs0 = time.perf_counter()
                pr = rag.submit_async([q for q, _ in queued], params)
                pr.t0 = [t for _, t in queued]        # latency counts the batching wait
                pending.append(pr)
                queued.clear()
                hostprof["submit"].append(time.perf_counter() - hs0)
            hostprof["poll"].append(hw1 - hw0)
            hostprof["work"].append(time.perf_counter() - hw0)
            st["ramping"] = st["ramping"] and clients[0] < R

        while len(out) < n_done:
            for req in llm.step(between=host_work):
                res = active.pop(req.id, None)
                if res is not None:
                    out.append(res)
                    clients[0] -= 1
                    if len(out) % R == 0:
                        progress(f"{st_name} {len(out) // R}/{n_done // R} ({time.time() - t_setup:.0f} s)")
            if not llm.has_work():
                host_work(block=True)
        return out

    if args.mode == "wave":
        for _ in range(args.warmup):
            one_step()
    else:
        closed_loop(max(1, args.warmup) * R, ramping=True, st_name="warmup")
    if not args.no_quiet_gc:
        from nv_genai_amd.utils.runtime import quiet_gc

        quiet_gc()
    world_barrier()
    prof = None
    if args.profile_dir and rank == 0:
        from torch.profiler import ProfilerActivity, profile

        prof = profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA])
        prof.__enter__()
    llm.stats.update({k: 0 if isinstance(v, int) else 0.0 for k, v in llm.stats.items()})
    llm._host_steps.clear()
    llm.bucket_hist.clear()
    llm.ntok_hist.clear()
    llm._step_events.clear()
    llm.step_timing = args.step_timing
    for v in hostprof.values():
        v.clear()
    for k in getattr(rag, "submit_host_s", {}):
        rag.submit_host_s[k] = 0.0
    from nv_genai_amd import ops

    # the timed window on the GPU timeline: marker kernels a kernel trace can be cut at
    # (scripts/summarize_prof.py: busy time and idle gaps of exactly this window)
    ops.region_marker(pctx.device, end=False)
    t0 = time.perf_counter()
    results = []
    if args.mode == "wave":
        for _ in range(args.steps):
            results += one_step()
    else:
        results = closed_loop(args.steps * R, ramping=False, st_name="timed")
    ops.region_marker(pctx.device, end=True)
    world_barrier()
    elapsed = time.perf_counter() - t0
    llm.stop_followers()
    if prof is not None:
        prof.__exit__(None, None, None)
        os.makedirs(args.profile_dir, exist_ok=True)
        prof.export_chrome_trace(os.path.join(args.profile_dir, "trace.json"))
        with open(os.path.join(args.profile_dir, "top_kernels.txt"), "w") as f:
            f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=40))
    t_max = pd.all_reduce_max(elapsed)
    per_replica = pd.all_gather_objects(round(R * args.steps / elapsed, 3))
    # after the run: the custom collectives' call counts and sticky timeout flag cover it
    devices = rank_devices(pctx) if world > 1 else None
    n_req = R * args.steps * replicas
    qps = n_req / t_max
    lat = sorted(r.latency for r in results)
    ttft = sorted(r.ttft for r in results)
    ptoks = [r.prompt_tokens for r in results]
    hit_tok = int(sum(r.request.cached_prefix for r in results))
    out_tok = sum(len(r.request.output_ids) for r in results) * replicas
    p50 = statistics.median(lat)
    p95 = lat[min(len(lat) - 1, int(0.95 * len(lat)))]
    line = {
        "metric": ("end-to-end RAG QPS + p50 latency, Llama-3-8B + arctic-embed-l, 1M-doc index"
                   if (args.model, args.embed_model, args.index_size) == ("llama3-8b", "arctic-embed-l", 1_000_000)
                   else f"end-to-end RAG QPS + p50 latency, {args.model} + {args.embed_model}, "
                        f"{args.index_size}-doc index"),
        "value": round(qps, 4),
        "unit": "requests/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000 * t_max / args.steps, 2),
        "higher_is_better": True,
        "scaling": "weak",
        # reference-equivalent stack (HF eager + torch brute-force search) measured on the
        # same MI355X: 4.40 QPS per GPU (BASELINE.md "Measured on MI355X")
        "vs_baseline": round(qps / (REF_EQUIV_QPS_PER_GPU * world), 3),
        "dtype": ("fp8-w8a8" if args.fp8 else "bf16") + (" + fp8 KV cache" if args.kv_fp8 else
                                                           (" (bf16 attention + KV)" if args.fp8 else "")),
        "data": f"synthetic: random-init weights; {args.index_size:,}-vector random unit-vector index + generated "
                "~500-token chunks; generated questions",
        "config": {
            "model": f"{args.model} + {args.embed_model}",
            "global_batch": R * replicas,
            "seq_len": int(statistics.mean(ptoks)) + args.max_tokens,
            "parallelism": f"dp{replicas}" + (f"xtp{tp}" if tp > 1 else ""),
            "sharded_index": sharded,
            "index_size": args.index_size,
            "top_k": args.top_k,
            "max_tokens": args.max_tokens,
            "concurrency_per_replica": R,
            "load": args.mode,
            "mixed_prefill_tokens": args.mixed_prefill_tokens,
        },
        "p50_latency_ms": round(1000 * p50, 1),
        "p95_latency_ms": round(1000 * p95, 1),
        "p50_ttft_ms": round(1000 * statistics.median(ttft), 1),
        "mean_prompt_tokens": round(statistics.mean(ptoks), 1),
        "output_tokens_per_s": round(out_tok / t_max, 1),
        "prefill_s": round(llm.stats["prefill_time"], 3),
        "decode_s": round(llm.stats["decode_time"], 3),
        "steps_prefill_decode_mixed": [llm.stats["prefill_steps"] - llm.stats["mixed_steps"],
                                       llm.stats["decode_steps"], llm.stats["mixed_steps"]],
        "unpipelined_steps": llm.stats["unpipelined_steps"],
        "submit_host_ms": {k: round(1e3 * v, 1) for k, v in getattr(rag, "submit_host_s", {}).items()},
        "host_work_ms": {k: [len(v), round(1e3 * sum(v), 1), round(1e3 * max(v), 2) if v else 0.0,
                             sum(1 for x in v if x > 4e-3)] for k, v in hostprof.items()},
        "host_s": {k[5:-2]: round(llm.stats[k], 3) for k in ("host_sched_s", "host_launch_s", "host_between_s",
                                                             "host_wait_s", "host_finalize_s")},
        "host_step_ms": host_step_summary(llm),
        **({"gpu_step_timing": llm.gpu_step_timing()} if args.step_timing and gpu else {}),
        "setup_s": round(setup_s, 1),
        "world_size": world,
        "backend": pctx.backend,
        "shared_devices": shared,
        **({"devices": devices} if devices else {}),
        "per_replica_qps": [x for x in per_replica if x is not None],
        "step_graphs": {"timed_graph_steps": llm.stats["graph_steps"],
                        "captured_total": len(llm.mgraphs),
                        "captured_in_timed_region": llm.stats["graph_captures"],
                        "capture_s_in_timed_region": round(llm.stats["graph_capture_s"], 3),
                        "launches_by_token_bucket": dict(sorted(llm.bucket_hist.items())),
                        "launches_by_tokens_128": dict(sorted(llm.ntok_hist.items()))},
        "prefix_cache_hit_blocks": int(llm.sched.prefix_hits()),
        # the timed requests' prompt tokens served from cached KV pages (skipped in prefill):
        # the share of prefill work the synthetic corpus's shared passages save
        "prefix_cache": {"enabled": bool(args.prefix_cache),
                         "hit_tokens": hit_tok, "prompt_tokens_total": sum(ptoks),
                         "hit_share": round(hit_tok / max(1, sum(ptoks)), 4)},
        **({"kv_page_refs_per_unique": round(llm.stats["kv_page_refs"] / max(1, llm.stats["kv_pages_unique"]), 4)}
           if llm.stats.get("kv_pages_unique") else {}),
        "distinct_docs_retrieved": len({d for r in results for d in r.doc_ids}),
    }
    if rank == 0:
        s = json.dumps(line)
        print(s, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(s + "\n")
        if args.timeline_out:
            with open(args.timeline_out, "w") as f:
                json.dump(llm.timeline(4096), f)
    pd.destroy()


if __name__ == "__main__":
    main()
