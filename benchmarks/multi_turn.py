"""Multi-turn RAG benchmark (BASELINE.json configs[2]: "Llama-3-8B + conversation-memory
retriever on 1 MI355X"; SURVEY.md §2.A C8, reference
RetrievalAugmentedGeneration/examples/multi_turn_rag/chains.py).

``--sessions`` concurrent chat sessions each run ``--turns`` turns. Every turn follows the
reference chain:
1. embed the question (query prefix);
2. top-k over the 1M-document index and over the shared ``conv_store`` memory index;
3. fill ``multi_turn_rag_template`` with {input}, {history} and {context};
4. generate the answer (Llama-3 chat template, exactly ``--max-tokens`` tokens);
5. write "User previously responded with ..." and "Agent previously responded with ..." back
   into ``conv_store``: embed both passages and insert them into the index and the docstore.

The memory index therefore grows while the benchmark runs. One retrieval worker owns the
encoder and both indexes and serves queued queries and memory writes in batches on its own
HIP stream; the LLM engine steps on its own thread (``EngineService``). Rank 0 prints one JSON line
with turns/s and the p50/p95 turn latency.
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

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--embed-model", default="arctic-embed-l")
    ap.add_argument("--index-size", type=int, default=1_000_000)
    ap.add_argument("--sessions", type=int, default=64)
    ap.add_argument("--turns", type=int, default=4)
    ap.add_argument("--warmup-sessions", type=int, default=8)
    ap.add_argument("--max-tokens", type=int, default=256)
    ap.add_argument("--top-k", type=int, default=4)
    ap.add_argument("--max-num-seqs", type=int, default=256)
    ap.add_argument("--out", default=None)
    return ap.parse_args(argv)


def main(argv=None):
    args = parse(argv)
    import torch

    from nv_genai_amd.chain_server.configuration import PromptsConfig
    from nv_genai_amd.engine.embed_engine import EmbeddingEngine
    from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine, SamplingParams
    from nv_genai_amd.index.docstore import DocStore, SyntheticDocStore
    from nv_genai_amd.index.flat import FlatIndex
    from nv_genai_amd.parallel import dist as pd
    from nv_genai_amd.serving.engine_service import EngineService
    from nv_genai_amd.utils.synthetic import TextGen

    pctx = pd.init_distributed(tp_size=1)
    gpu = pctx.device.type == "cuda"
    dev = str(pctx.device)
    t0 = time.time()
    eng = LLMEngine(EngineConfig(model=args.model, max_num_seqs=args.max_num_seqs, max_batched_tokens=16384,
                                 max_model_len=8192, use_graphs=gpu, kv_cache_blocks=None if gpu else 512,
                                 seed=pctx.rank), device=dev, pctx=pctx)
    emb = EmbeddingEngine(args.embed_model, device=dev, seed=pctx.rank)
    docs_index = FlatIndex(emb.dim, "cosine", dev, capacity=args.index_size)
    docs_index.add_random(args.index_size, seed=1234)
    docs = SyntheticDocStore(args.index_size)
    conv_index = FlatIndex(emb.dim, "cosine", dev, capacity=1 << 16)
    conv_docs = DocStore()
    lock = threading.Lock()
    template = PromptsConfig().multi_turn_rag_template
    tok = eng.tok
    svc = EngineService(eng)
    params = SamplingParams(temperature=0.2, top_p=0.7, max_tokens=args.max_tokens, ignore_eos=True)
    setup_s = time.time() - t0
    stats = {"prompt_tokens": 0, "output_tokens": 0, "history_hits": 0}
    ttft = []

    # One retrieval worker owns the encoder and both indexes: it drains queued memory writes
    # and queries in batches on its own HIP stream, so retrieval neither queues behind the
    # engine's in-flight step nor serialises the sessions one GPU round-trip at a time.
    import concurrent.futures as cf
    import queue as _queue

    work: "_queue.Queue" = _queue.Queue()
    rstream = torch.cuda.Stream(device=dev) if gpu else None

    def retrieval_worker():
        while True:
            items = [work.get()]
            if items[0] is None:
                return
            time.sleep(0.002)                      # let a batch form
            while True:
                try:
                    items.append(work.get_nowait())
                except _queue.Empty:
                    break
            stop = any(it is None for it in items)
            items = [it for it in items if it is not None]
            writes = [it for it in items if it[0] == "write"]
            reads = [it for it in items if it[0] == "read"]
            try:
                serve(writes, reads)
            except BaseException as e:  # noqa: BLE001 - fail the waiting turns, never hang them
                for it in writes + reads:
                    if not it[2].done():
                        it[2].set_exception(e)
            if stop:
                return

    def serve(writes, reads):
            ctxmgr = torch.cuda.stream(rstream) if gpu else _nullctx()
            with ctxmgr:
                if writes:
                    texts = [t for w in writes for t in w[1]]
                    v = emb.embed(texts, input_type="passage")
                    new = conv_docs.new_ids(len(texts))
                    conv_docs.add(new, texts)
                    conv_index.add(v, torch.tensor(new))
                    for w in writes:
                        w[2].set_result(None)
                if reads:
                    q = emb.embed([r[1] for r in reads], input_type="query")
                    _, di = docs_index.search(q, args.top_k)
                    hi = conv_index.search(q, args.top_k)[1] if len(conv_index) else None
                    di = di.cpu().tolist()
                    hi = None if hi is None else hi.cpu().tolist()
                    for j, r in enumerate(reads):
                        ctx = "".join(docs.get(int(i)) + "\n\n" for i in di[j] if int(i) >= 0)
                        hist = "" if hi is None else "".join(conv_docs.get(int(i)) + "\n\n" for i in hi[j] if int(i) >= 0)
                        r[2].set_result((ctx, hist, 0 if hi is None else sum(int(i) >= 0 for i in hi[j])))

    worker = threading.Thread(target=retrieval_worker, daemon=True)
    worker.start()

    def turn(question: str) -> float:
        t = time.perf_counter()
        fut = cf.Future()
        work.put(("read", question, fut))
        ctx, hist, nh = fut.result()
        prompt = (template.replace("{input}", question).replace("{history}", hist)
                  .replace("{context}", ctx)) + "User Query: " + question
        ids = tok.apply_chat_template([{"role": "user", "content": prompt}])
        h = svc.submit(ids, params)
        answer = h.text()
        r = h.request
        mem = [f"User previously responded with {question}", f"Agent previously responded with {answer}"]
        wf = cf.Future()
        work.put(("write", mem, wf))
        wf.result()                                # the next turn sees this turn's memory
        with lock:
            stats["prompt_tokens"] += len(ids)
            stats["output_tokens"] += len(r.output_ids)
            stats["history_hits"] += nh
            if r.ttft is not None:
                ttft.append(r.ttft)
        return time.perf_counter() - t

    def session(seed: int):
        gen = TextGen(seed=seed)
        return [turn(gen.question()) for _ in range(args.turns)]

    def run(n: int, seed0: int):
        with ThreadPoolExecutor(max_workers=n) as ex:
            return [x for lat in ex.map(session, range(seed0, seed0 + n)) for x in lat]

    if args.warmup_sessions:
        run(args.warmup_sessions, 50_000 + 1000 * pctx.rank)
    for k in stats:
        stats[k] = 0
    ttft.clear()
    pd.barrier()
    t1 = time.perf_counter()
    lat = run(args.sessions, 1000 * pctx.rank)
    elapsed = time.perf_counter() - t1
    t_max = pd.all_reduce_max(elapsed)
    svc.shutdown()
    work.put(None)
    worker.join(timeout=30)
    n_turns = args.sessions * args.turns * pctx.world_size
    lat.sort()
    res = {"metric": "multi-turn RAG turns/s + p50 latency (conversation-memory retriever)",
           "value": round(n_turns / t_max, 4), "unit": "turns/s", "n_gpus": pctx.world_size if gpu else 0,
           "parallelism": f"dp{pctx.world_size}", "model": args.model, "embed_model": args.embed_model,
           "index_size": args.index_size, "sessions_per_gpu": args.sessions, "turns": args.turns,
           "elapsed_s": round(t_max, 3), "p50_latency_ms": round(1e3 * statistics.median(lat), 1),
           "p95_latency_ms": round(1e3 * lat[min(len(lat) - 1, int(0.95 * len(lat)))], 1),
           "p50_ttft_ms": round(1e3 * statistics.median(ttft), 1) if ttft else None,
           "mean_prompt_tokens": round(stats["prompt_tokens"] / max(1, len(lat)), 1),
           "memory_entries": len(conv_index), "history_hits_per_turn": round(stats["history_hits"] / max(1, len(lat)), 2),
           "output_tokens_per_s": round(stats["output_tokens"] * pctx.world_size / t_max, 1),
           "dtype": "bf16", "data": "synthetic: random-init weights, random unit-vector index, generated questions",
           "setup_s": round(setup_s, 1)}
    if pctx.rank == 0:
        line = json.dumps(res)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")
    pd.destroy()


if __name__ == "__main__":
    main()
