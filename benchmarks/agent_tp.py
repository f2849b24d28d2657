"""Query-decomposition agent benchmark (BASELINE.json configs[3]: "Llama-3-70B TP=8 over xGMI
+ 10M-vec index sharded across 8 GPUs").

One model-parallel replica over every rank of the job (``tp = world``): the driver (rank 0)
runs the agents, the LLM engine's scheduler and the query encoder; every rank holds 1/world
of the Llama weights and KV heads, and 1/world of the index. A sub-question's retrieval is a
command on the replica's step channel (``LLMEngine.broadcast_command``), executed on the
engine thread between steps (``EngineService.call``): the query block is broadcast, each rank
scores its shard with the MFMA score + top-k kernels, the per-shard top-k lists are
all-gathered and merged.

The weights are random, so the agent follows the reference's trajectory with its decisions
scripted (``--sub-questions`` sub-questions answered by Search, then Nil) while every LLM
call keeps its real prompt and a fixed output length:

1. decomposition prompt (reference TEMPLATE + ledger) -> ``--plan-tokens`` tokens;
2. per sub-question: embed -> sharded top-4 -> extract-answer prompt with the 4 passages
   -> ``--extract-tokens`` tokens;
3. a second decomposition round with the filled ledger (-> Nil);
4. the final answer prompt (question + sub-answers) -> ``--answer-tokens`` tokens.

``--concurrency`` agents run at once; the line printed by rank 0 reports agent queries/s,
p50/p95 latency and LLM calls/s. Examples::

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/agent_tp.py      # 70B TP=8, 10M
    python benchmarks/agent_tp.py --model llama3-70b --index-size 10000000          # 1 GPU, 70B fits
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SEARCH_CMD = -3


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--embed-model", default="arctic-embed-l")
    ap.add_argument("--index-size", type=int, default=10_000_000)
    ap.add_argument("--queries", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--concurrency", type=int, default=32)
    ap.add_argument("--sub-questions", type=int, default=2)
    ap.add_argument("--plan-tokens", type=int, default=48)
    ap.add_argument("--extract-tokens", type=int, default=48)
    ap.add_argument("--answer-tokens", type=int, default=256)
    ap.add_argument("--top-k", type=int, default=4)
    ap.add_argument("--max-num-seqs", type=int, default=128)
    ap.add_argument("--kv-cache-fraction", type=float, default=0.5)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--fp8", action="store_true", help="W8A8 FP8 projections (70B: 70 GB of weights)")
    ap.add_argument("--search-legacy", action="store_true",
                    help="A/B: the round-5 search path (query block broadcast as its own collective, "
                         "results gathered over the process group) instead of queries in the step-channel "
                         "command + the IPC all-gather")
    ap.add_argument("--out", default=None)
    return ap.parse_args(argv)


def main(argv=None, emit: bool = True, record_devices=None):
    """Run the benchmark; the driver returns the result dict (and prints it when ``emit``),
    follower ranks return None. ``record_devices(pctx)``: a collective run-record hook called
    on every rank right after the process group exists (bench.py's per-rank device record)."""
    args = parse(argv)
    from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine, SamplingParams
    from nv_genai_amd.examples.query_decomposition_rag.chains import EXTRACT_PROMPT, TEMPLATE, Ledger
    from nv_genai_amd.index.sharded import ShardedIndex
    from nv_genai_amd.parallel import dist as pd

    pctx = pd.init_distributed(tp_size=int(os.environ.get("WORLD_SIZE", "1")))
    devices = record_devices(pctx) if record_devices is not None else None
    gpu = pctx.device.type == "cuda"
    dev = str(pctx.device)
    t0 = time.time()
    eng = LLMEngine(EngineConfig(model=args.model, max_num_seqs=args.max_num_seqs, max_batched_tokens=16384,
                                 max_model_len=8192, kv_cache_fraction=args.kv_cache_fraction,
                                 use_graphs=gpu and not args.no_graphs, kv_cache_blocks=None if gpu else 512,
                                 fp8=args.fp8),
                    device=dev, pctx=pctx)
    from nv_genai_amd.models.config import encoder_config

    dim = encoder_config(args.embed_model).hidden
    index = ShardedIndex(dim, "cosine", dev, pctx=pctx, group=pctx.mp_group if pctx.mp_size > 1 else None,
                         capacity=max(1024, args.index_size // max(1, pctx.world_size) + 1),
                         ipc_gather=not args.search_legacy)
    index.add_random(args.index_size, seed=1234)
    k = args.top_k
    if not eng.is_driver:
        comm_dev = index.comm_dev
        def search_hook(n, payload=None):
            if payload is not None:   # the driver's query block, from the command: side stream
                return index.search_side(payload, n, k, wait=False)
            return index.search(torch.zeros(n, dim, device=comm_dev), k)
        eng.run_follower(hooks={SEARCH_CMD: search_hook})
        pd.destroy()
        return None

    import jinja2

    from nv_genai_amd.engine.embed_engine import EmbeddingEngine
    from nv_genai_amd.index.docstore import SyntheticDocStore
    from nv_genai_amd.serving.engine_service import EngineService
    from nv_genai_amd.utils.synthetic import TextGen

    emb = EmbeddingEngine(args.embed_model, device=dev)
    emb_lock = threading.Lock()
    docs = SyntheticDocStore(args.index_size)
    tok = eng.tok
    svc = EngineService(eng)
    tmpl = jinja2.Environment().from_string(TEMPLATE)
    setup_s = time.time() - t0
    stats = {"llm_calls": 0, "searches": 0, "prompt_tokens": 0, "output_tokens": 0}
    search_ms = []
    slock = threading.Lock()

    def llm(prompt: str, max_tokens: int) -> str:
        ids = tok.apply_chat_template([{"role": "user", "content": prompt}])
        h = svc.submit(ids, SamplingParams(temperature=0.2, top_p=0.7, max_tokens=max_tokens, ignore_eos=True))
        out = h.text()
        with slock:
            stats["llm_calls"] += 1
            stats["prompt_tokens"] += len(ids)
            stats["output_tokens"] += len(h.request.output_ids)
        return out

    def retrieve(question: str):
        with emb_lock:
            q = emb.embed([question], input_type="query")
        qv = q.to(index.comm_dev if not gpu else dev).float()

        def run():
            # on the engine thread, between steps: every rank of the replica joins
            t = time.perf_counter()
            if index.world == 1:
                out = index.search(qv, k)
            elif args.search_legacy:
                eng.broadcast_command(SEARCH_CMD, qv.shape[0])
                out = index.search(qv, k)
            else:
                # the query block rides in the command: the search's only collective is the
                # packed (score, id) all-gather, on the index's own stream on every rank
                payload = index.query_payload(qv)
                eng.broadcast_command(SEARCH_CMD, qv.shape[0], payload)
                out = index.search_side(payload.view(np.uint8).reshape(-1), qv.shape[0], k)
            ids = out[1].cpu()
            search_ms.append(1e3 * (time.perf_counter() - t))
            return ids
        ids = svc.call(run).result()
        with slock:
            stats["searches"] += 1
        return [docs.get(int(i)) for i in ids[0].tolist() if int(i) >= 0]

    def agent(question: str, gen: TextGen) -> float:
        t = time.perf_counter()
        ledger = Ledger()
        llm(tmpl.render(context="", question=question), args.plan_tokens)
        for _ in range(args.sub_questions):          # scripted: Search with generated sub-questions
            sq = gen.question()
            chunks = retrieve(sq)
            p = EXTRACT_PROMPT + "Question: " + sq + "\n\n"
            for i, c in enumerate(chunks):
                p += f"Passage {i + 1}:\n{c}\n"
            ledger.question_trace.append(sq)
            ledger.answer_trace.append(llm(p, args.extract_tokens))
        llm(tmpl.render(context=ledger.context().strip("\n"), question=question), args.plan_tokens)  # -> Nil
        final = "Question: " + question + "\n\nSub Questions and Answers\n"
        for q_, a_ in zip(ledger.question_trace, ledger.answer_trace):
            final += f"Sub Question: {q_}\nSub Answer: {a_}\n"
        llm(final + "\nFinal Answer: ", args.answer_tokens)
        return time.perf_counter() - t

    def run(n: int, seed: int):
        gens = [TextGen(seed=seed + i) for i in range(n)]
        with ThreadPoolExecutor(max_workers=args.concurrency) as ex:
            return list(ex.map(lambda g: agent(g.question(), g), gens))

    if args.warmup:
        run(args.warmup, 10_000)
    for key in stats:
        stats[key] = 0
    search_ms.clear()
    t1 = time.perf_counter()
    lat = run(args.queries, 20_000)
    elapsed = time.perf_counter() - t1
    svc.shutdown()
    eng.stop_followers()
    lat.sort()
    res = {"metric": "query-decomposition agent QPS + p50 latency (scripted trajectory)",
           "value": round(args.queries / elapsed, 4), "unit": "agent queries/s",
           "n_gpus": pctx.world_size if gpu else 0, "parallelism": f"tp{pctx.tp_size}",
           "model": args.model, "embed_model": args.embed_model, "index_size": args.index_size,
           "concurrency": args.concurrency, "queries": args.queries, "elapsed_s": round(elapsed, 3),
           "search_path": "legacy" if args.search_legacy else "command-payload+ipc-gather",
           "p50_latency_ms": round(1e3 * statistics.median(lat), 1),
           "p95_latency_ms": round(1e3 * lat[min(len(lat) - 1, int(0.95 * len(lat)))], 1),
           "llm_calls_per_s": round(stats["llm_calls"] / elapsed, 2),
           "searches_per_s": round(stats["searches"] / elapsed, 2),
           "mean_prompt_tokens": round(stats["prompt_tokens"] / max(1, stats["llm_calls"]), 1),
           "output_tokens_per_s": round(stats["output_tokens"] / elapsed, 1),
           "dtype": "fp8-w8a8" if args.fp8 else "bf16",
           "data": "synthetic: random-init weights, random unit-vector index, generated questions",
           "setup_s": round(setup_s, 1), "backend": pctx.backend,
           "search": {**{k_: v for k_, v in index.stats.items() if k_ != "host_s"},
                      "host_ms_per_search": round(1e3 * index.stats["host_s"] / max(1, index.stats["searches"]), 3),
                      **({"p50_ms": round(sorted(search_ms)[len(search_ms) // 2], 3),
                          "p95_ms": round(sorted(search_ms)[int(0.95 * (len(search_ms) - 1))], 3)}
                         if search_ms else {})},
           **({"devices": devices} if devices else {})}
    line = json.dumps(res)
    if emit:
        print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    pd.destroy()
    return res


if __name__ == "__main__":
    main()
