#!/usr/bin/env python3
"""Decode-step microbenchmark of the LLM engine: B sequences at context length L, timed
engine.step() (scheduler + graph replay + sampling + host sync) and bare graph replay.
Prints one JSON line; with --prefill also times a batched prefill of the same prompts."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--ctx", type=int, default=1400)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--shared-prefix", type=int, default=0,
                    help="every prompt starts with the same N tokens (prefix cache on): the RAG "
                         "template case of the shared-prefix decode pass")
    args = ap.parse_args()
    from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine, SamplingParams

    B, L = args.batch, args.ctx
    eng = LLMEngine(EngineConfig(model=args.model, max_num_seqs=B, max_batched_tokens=32768,
                                 max_model_len=8192, use_graphs=not args.no_graphs,
                                 graph_batch_sizes=(B,), enable_prefix_caching=args.shared_prefix > 0,
                                 mixed_prefill_tokens=0, token_alignment=1))
    g = torch.Generator().manual_seed(0)
    V = 30000
    P = min(args.shared_prefix, L - 1)
    head = torch.randint(100, V, (P,), generator=g).tolist()
    prompts = [head + torch.randint(100, V, (L - P,), generator=g).tolist() for _ in range(B)]
    p = SamplingParams(temperature=0.7, top_p=0.9, max_tokens=args.steps + 64, ignore_eos=True)
    reqs = []
    if P:   # the first prompt fills the prefix cache; the rest find its pages
        reqs.append(eng.add_request(prompts[0], p))
        while len(reqs[0].output_ids) == 0:
            eng.step()
    reqs += [eng.add_request(x, p) for x in prompts[len(reqs):]]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while any(len(r.output_ids) == 0 for r in reqs):
        eng.step()
    torch.cuda.synchronize()
    t_prefill = time.perf_counter() - t0
    for _ in range(3):
        eng.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.step()
    torch.cuda.synchronize()
    t_step = (time.perf_counter() - t0) / args.steps
    t_replay = None
    if eng.graphs:
        gr = eng.graphs[B]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            gr.replay()
        torch.cuda.synchronize()
        t_replay = (time.perf_counter() - t0) / args.steps
    cfg = eng.mcfg
    wbytes = cfg.num_params() * 2
    kvbytes = B * (L + 4) * cfg.kv_bytes_per_token()
    out = {"model": args.model, "batch": B, "ctx": L, "prefill_s": round(t_prefill, 3),
           "prefill_tok_s": round(B * L / t_prefill), "step_ms": round(1000 * t_step, 3),
           "replay_ms": None if t_replay is None else round(1000 * t_replay, 3),
           "decode_tok_s": round(B / t_step), "weights_GB": round(wbytes / 1e9, 2),
           "kv_GB": round(kvbytes / 1e9, 2),
           "eff_TBps": round((wbytes + kvbytes) / (t_replay or t_step) / 1e12, 3),
           "shared_prefix": P}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
