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
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch


REF_EQUIV_QPS_PER_GPU = 4.40   # profiles/r1_refeq/ref_eq.json


def parse():
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
    ap.add_argument("--step-timing", action="store_true",
                    help="GPU events around every engine step: in-step time vs idle between steps")
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
    return ap.parse_args()


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


def main():
    args = parse()
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
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

    pctx = pd.init_distributed(tp_size=1)
    world, rank = pctx.world_size, pctx.rank
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
    ecfg = EngineConfig(model=args.model, max_num_seqs=max(R, 1), max_batched_tokens=args.max_batched_tokens,
                        max_model_len=8192, use_graphs=gpu and not args.no_graphs,
                        graph_batch_sizes=sizes, seed=rank, kv_cache_fraction=0.3,
                        mixed_prefill_tokens=args.mixed_prefill_tokens,
                        mixed_min_tokens=args.mixed_min_tokens, mixed_max_wait=args.mixed_max_wait,
                        fp8=args.fp8, kv_cache_dtype="fp8" if args.kv_fp8 else "auto")
    llm = LLMEngine(ecfg, device=dev, pctx=pctx)
    emb = EmbeddingEngine(args.embed_model, device=dev, seed=rank)
    index = FlatIndex(emb.dim, "cosine", dev, capacity=args.index_size)
    index.add_random(args.index_size, seed=1234)
    docs = SyntheticDocStore(args.index_size)
    rag = RAGPipeline(llm, emb, index, docs, top_k=args.top_k)
    gen = TextGen(seed=100 + rank)
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

    def closed_loop(n_done: int, ramping: bool):
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
            if not llm.has_work():
                host_work(block=True)
        return out

    if args.mode == "wave":
        for _ in range(args.warmup):
            one_step()
    else:
        closed_loop(max(1, args.warmup) * R, ramping=True)
    if not args.no_quiet_gc:
        from nv_genai_amd.utils.runtime import quiet_gc

        quiet_gc()
    pd.barrier()
    if gpu:
        torch.cuda.synchronize()
    prof = None
    if args.profile_dir and rank == 0:
        from torch.profiler import ProfilerActivity, profile

        prof = profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA])
        prof.__enter__()
    llm.stats.update({k: 0 if isinstance(v, int) else 0.0 for k, v in llm.stats.items()})
    llm._host_steps.clear()
    llm._step_events.clear()
    llm.step_timing = args.step_timing
    for v in hostprof.values():
        v.clear()
    t0 = time.perf_counter()
    results = []
    if args.mode == "wave":
        for _ in range(args.steps):
            results += one_step()
    else:
        results = closed_loop(args.steps * R, ramping=False)
    if gpu:
        torch.cuda.synchronize()
    pd.barrier()
    elapsed = time.perf_counter() - t0
    if prof is not None:
        prof.__exit__(None, None, None)
        os.makedirs(args.profile_dir, exist_ok=True)
        prof.export_chrome_trace(os.path.join(args.profile_dir, "trace.json"))
        with open(os.path.join(args.profile_dir, "top_kernels.txt"), "w") as f:
            f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=40))
    t_max = pd.all_reduce_max(elapsed)
    n_req = R * args.steps * world
    qps = n_req / t_max
    lat = sorted(r.latency for r in results)
    ttft = sorted(r.ttft for r in results)
    ptoks = [r.prompt_tokens for r in results]
    out_tok = sum(len(r.request.output_ids) for r in results) * world
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
        "data": "synthetic: random-init weights; 1M random unit-vector index + generated ~500-token chunks; generated questions",
        "config": {
            "model": f"{args.model} + {args.embed_model}",
            "global_batch": R * world,
            "seq_len": int(statistics.mean(ptoks)) + args.max_tokens,
            "parallelism": f"dp{world}",
            "index_size": args.index_size,
            "top_k": args.top_k,
            "max_tokens": args.max_tokens,
            "concurrency_per_gpu": R,
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
        "host_work_ms": {k: [len(v), round(1e3 * sum(v), 1), round(1e3 * max(v), 2) if v else 0.0,
                             sum(1 for x in v if x > 4e-3)] for k, v in hostprof.items()},
        "host_s": {k[5:-2]: round(llm.stats[k], 3) for k in ("host_sched_s", "host_launch_s", "host_between_s",
                                                             "host_wait_s", "host_finalize_s")},
        "host_step_ms": host_step_summary(llm),
        **({"gpu_step_timing": llm.gpu_step_timing()} if args.step_timing and gpu else {}),
        "setup_s": round(setup_s, 1),
        "prefix_cache_hit_blocks": int(llm.sched.prefix_hits()),
        "distinct_docs_retrieved": len({d for r in results for d in r.doc_ids}),
    }
    if rank == 0:
        s = json.dumps(line)
        print(s, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(s + "\n")
    pd.destroy()


if __name__ == "__main__":
    main()
