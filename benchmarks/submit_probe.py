"""Does retrieval submission wait for the GPU? (host-side probe, bench.py's host_work path)

The headline bench calls ``RAGPipeline.submit_async`` between launching an engine step and
waiting for it. If anything in the query embedding or search path synchronises with the
device, the host blocks until the in-flight step finishes and the next step launches late.

This probe keeps the main stream busy with a spin kernel of known length and times each
piece of the submission path (tokenise, embed, search, pinned copies) on the retrieval
stream. A piece that takes about the spin time is waiting for the main stream.
Usage: python benchmarks/submit_probe.py [--embed-model arctic-embed-l] [--index-size N]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--embed-model", default="arctic-embed-l")
    ap.add_argument("--index-size", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--spin-ms", type=float, default=40.0)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    from nv_genai_amd.engine.embed_engine import EmbeddingEngine
    from nv_genai_amd.index.flat import FlatIndex
    from nv_genai_amd.utils.synthetic import TextGen

    dev = "cuda:0"
    emb = EmbeddingEngine(args.embed_model, device=dev)
    idx = FlatIndex(emb.dim, "cosine", dev, capacity=args.index_size)
    idx.add_random(args.index_size, seed=1234)
    gen = TextGen(seed=5)
    emb.calibrate_whitening([gen.question() for _ in range(2048)])
    side = torch.cuda.Stream(dev)
    # spin-kernel cycles per ms (calibrated once)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(10_000_000)
    e1.record()
    torch.cuda.synchronize()
    cyc_per_ms = 10_000_000 / e0.elapsed_time(e1)

    def run(spin: bool):
        qs = [gen.question() for _ in range(args.batch)]
        torch.cuda.synchronize()
        if spin:
            torch.cuda._sleep(int(cyc_per_ms * args.spin_ms))
        t = {"t0": time.perf_counter()}
        with torch.cuda.stream(side):
            seqs = emb.tokenize(qs, "query")
            t["tokenize"] = time.perf_counter()
            q = emb.embed_ids(seqs)
            t["embed"] = time.perf_counter()
            s, i = idx.search(q, 4)
            t["search"] = time.perf_counter()
            hs = torch.empty(s.shape, dtype=s.dtype, pin_memory=True)
            hi = torch.empty(i.shape, dtype=i.dtype, pin_memory=True)
            t["pin_alloc"] = time.perf_counter()
            hs.copy_(s, non_blocking=True)
            hi.copy_(i, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(side)
            t["copy"] = time.perf_counter()
        ev.synchronize()
        t["side_done"] = time.perf_counter()
        torch.cuda.synchronize()
        keys = list(t)
        return {k: round((t[k] - t[p]) * 1e3, 3) for p, k in zip(keys, keys[1:])}

    for _ in range(3):
        run(False)
    res = {"spin_ms": args.spin_ms, "batch": args.batch}
    for spin in (False, True):
        rows = [run(spin) for _ in range(args.reps)]
        res["spin" if spin else "idle"] = {k: round(sorted(r[k] for r in rows)[len(rows) // 2], 3) for k in rows[0]}
    # sync-debug pass: which torch ops synchronise
    torch.cuda.set_sync_debug_mode("warn")
    run(True)
    torch.cuda.set_sync_debug_mode(0)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
