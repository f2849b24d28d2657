"""Streaming-ingest throughput (reference
experimental/streaming_ingest_rag vdb_upload pipeline: file source -> chunker -> Triton
all-MiniLM-L6-v2 (TensorRT FP16, max_batch 256, seq 512) -> vector-DB writer, with MonitorStage
rates; the reference publishes no rate).

``--docs`` synthetic ~4 KB text files go through ``ingest.streaming.IngestPipeline`` with the
reference pipeline settings: 512-character chunks, pipeline_batch_size 1024, max_batch_size
256, edge_buffer_size 128, writer batch 5120. The stages are the filesystem source, the chunker
threads, micro-batched GPU embedding on the HIP encoder, and the in-HBM vector-store writer.
Prints the rate of each stage and the end-to-end chunks/s.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=2000)
    ap.add_argument("--embed-model", default="all-minilm-l6-v2")
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)
    import torch

    from nv_genai_amd.engine.embed_engine import EmbeddingEngine
    from nv_genai_amd.index.vectorstore import VectorStore
    from nv_genai_amd.ingest.streaming import IngestPipeline
    from nv_genai_amd.utils.synthetic import TextGen

    dev = "cuda" if torch.cuda.is_available() else "cpu"
    emb = EmbeddingEngine(args.embed_model, device=dev)
    gen = TextGen(seed=5)
    stores = {}
    with tempfile.TemporaryDirectory() as d:
        for i in range(args.docs):
            with open(os.path.join(d, f"doc{i:05d}.txt"), "w") as f:
                f.write(" ".join(gen.paragraph((8, 12)) for _ in range(3)))
        cfg = {"vdb_pipeline": {
            "pipeline": {"edge_buffer_size": 128, "max_batch_size": 256, "num_threads": args.threads,
                         "pipeline_batch_size": 1024, "chunk_size": 512, "chunk_overlap": 51},
            "vdb": {"batch_size": 5120, "resource_name": "VDBGENERAL"},
            "sources": [{"type": "filesystem", "name": "files",
                         "config": {"filenames": [os.path.join(d, "*.txt")]}}]}}

        def factory(name, recreate):
            stores[name] = VectorStore(emb, emb.dim, name=name, device=dev, batch_queries=False)
            return stores[name]

        emb.embed(["warm up"] * 8, input_type="passage")       # kernels resident before timing
        t0 = time.perf_counter()
        mons = IngestPipeline(cfg, emb, factory).run()
        if dev == "cuda":
            torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
    chunks = mons["upload"].count
    res = {"metric": "streaming ingest throughput (file -> chunk -> GPU embed -> in-HBM index)",
           "value": round(chunks / elapsed, 1), "unit": "chunks/s", "docs": args.docs, "chunks": chunks,
           "elapsed_s": round(elapsed, 3), "embed_model": args.embed_model, "device": dev,
           "stage_rates": {k: round(m.rate(), 1) for k, m in mons.items()},
           "indexed": sum(len(s) for s in stores.values())}
    line = json.dumps(res)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
