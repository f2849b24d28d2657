"""Embedding / reranking throughput against the reference's published encode rate.

The reference's only embedding number is from
experimental/synthetic-data-retriever-customization/retriever_customization.ipynb#cell 17-18:
a Megatron-SBERT encoder (NV-Embed-QA-4, BERT-large class) encodes 300 "query: ..." texts at
batch 5 at 32.25 it/s, and 100 "passage: ..." texts at batch 5 at 10.48 it/s. Its ``encode_text``
tokenises every text first, then times only the batched forwards.

This script follows the same protocol with the arctic-embed-l-shaped encoder (24 layers,
hidden 1024, random init) on the HIP kernels:
* batch 5, queries (generated questions) and ~500-token passages: it/s, where one it is one
  batch of 5;
* the serving envelopes: the Triton embedder (max_batch 256, seq 512,
  all-MiniLM-L6-v2_config.pbtxt) and the reranker (max_shapes [64, 512],
  nv-rerank-qa-mistral-4b-A6000.yaml), in texts/s.

The timed region covers forward + pooling + normalisation, and a device sync per batch (the
reference's tqdm loop blocks the same way). Tokenisation is outside it, as in the reference.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

REF_ITS = {"query_b5": 32.25, "passage_b5": 10.48}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="arctic-embed-l")
    ap.add_argument("--reranker", default="bge-reranker-large")
    ap.add_argument("--queries", type=int, default=300)
    ap.add_argument("--passages", type=int, default=100)
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)
    import torch

    from nv_genai_amd.engine.embed_engine import EmbeddingEngine
    from nv_genai_amd.utils.synthetic import TextGen

    dev = "cuda" if torch.cuda.is_available() else "cpu"
    emb = EmbeddingEngine(args.model, device=dev)
    gen = TextGen(seed=3)
    queries = [gen.question() for _ in range(args.queries)]
    passages = [" ".join(gen.paragraph((12, 18)) for _ in range(2)) for _ in range(args.passages)]
    q_ids = emb.tokenize(queries, "query")
    p_ids = emb.tokenize(passages, "passage")

    def sync():
        if dev == "cuda":
            torch.cuda.synchronize()

    def rate(seqs, bs, reps=3):
        for i in range(0, min(len(seqs), 4 * bs), bs):    # warm-up
            emb.embed_ids(seqs[i:i + bs])
        sync()
        best = 0.0
        for _ in range(reps):
            t = time.perf_counter()
            n = 0
            for i in range(0, len(seqs), bs):
                emb.embed_ids(seqs[i:i + bs])
                sync()
                n += 1
            best = max(best, n / (time.perf_counter() - t))
        return best

    out = {"model": args.model, "device": dev, "dtype": "bf16",
           "mean_query_tokens": round(sum(map(len, q_ids)) / len(q_ids), 1),
           "mean_passage_tokens": round(sum(map(len, p_ids)) / len(p_ids), 1)}
    out["query_b5_it_per_s"] = round(rate(q_ids, 5), 1)
    out["passage_b5_it_per_s"] = round(rate(p_ids, 5), 1)
    out["vs_reference_query_b5"] = round(out["query_b5_it_per_s"] / REF_ITS["query_b5"], 1)
    out["vs_reference_passage_b5"] = round(out["passage_b5_it_per_s"] / REF_ITS["passage_b5"], 1)
    big = (p_ids * (256 // len(p_ids) + 1))[:256]
    out["passage_b256_texts_per_s"] = round(256 * rate(big, 256, reps=2), 1)
    rr = EmbeddingEngine(args.reranker, device=dev)
    pairs = [rr.tok.encode_pair(queries[i % len(queries)], passages[i % len(passages)]) for i in range(64)]
    for _ in range(2):
        rr.embed_ids(pairs)
    sync()
    t = time.perf_counter()
    for _ in range(5):
        rr.embed_ids(pairs)
        sync()
    out["rerank_64x512_pairs_per_s"] = round(5 * 64 / (time.perf_counter() - t), 1)
    out["reference"] = {"query_b5_it_per_s": 32.25, "passage_b5_it_per_s": 10.48,
                        "source": "retriever_customization.ipynb#cell 18 (NV-Embed-QA-4, GPU unspecified)"}
    line = json.dumps(out)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
