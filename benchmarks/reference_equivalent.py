#!/usr/bin/env python3
"""Reference-equivalent RAG stack on the same MI355X, for the comparison BASELINE.md promises.

The reference publishes no number for its headline metric, so
per SURVEY.md §6 "Implication" we measure what a user of the reference gets when its GPU
services are replaced by the plain PyTorch building blocks the reference itself reaches for
when it runs models locally:

* LLM: HF-transformers ``LlamaForCausalLM`` (Llama-3-8B architecture, random init, bf16,
  ``sdpa`` attention) driven by ``model.generate`` with static batches — the reference's
  local-LLM path (examples/multimodal_rag/llm/llm.py:39-59, notebooks/02_Option(2)
  ``HuggingFacePipeline``);
* embedder: HF-transformers ``BertModel`` with arctic-embed-l dimensions, CLS pooling +
  L2-normalise (utils.py:294-309 runs ``HuggingFaceEmbeddings`` on ``cuda:0``);
* index: brute-force ``torch.topk(q @ X.T)`` over 1M x 1024 bf16 vectors in HBM (stands in
  for FAISS ``IndexFlatL2``/Milvus GPU_IVF_FLAT, utils.py:198-217 — and is faster than both).

The workload is the one ``bench.py`` serves: the same synthetic corpus, questions, top-4
retrieval, 1500-token context cap, reference ``rag_template`` + Llama-3 chat template
(built with the same ``RAGPipeline.build_prompt``), temperature 0.2 / top_p 0.7, exactly
``--max-tokens`` generated tokens per request (``min_new_tokens`` = ``max_new_tokens``).
Every batch is served end to end (embed -> search -> prompt -> generate); QPS = requests /
wall time. Prints one JSON line per batch size and a summary line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="64,128,256")
    ap.add_argument("--max-tokens", type=int, default=256)
    ap.add_argument("--index-size", type=int, default=1_000_000)
    ap.add_argument("--layers", type=int, default=None, help="debug only: fewer decoder layers")
    ap.add_argument("--out", default=None)
    ap.add_argument("--device", default="cuda")
    args = ap.parse_args()

    from transformers import BertConfig, BertModel, LlamaConfig, LlamaForCausalLM

    from nv_genai_amd.index.docstore import SyntheticDocStore
    from nv_genai_amd.models.config import encoder_config, llama_config
    from nv_genai_amd.rag.pipeline import RAGPipeline
    from nv_genai_amd.utils.synthetic import TextGen
    from nv_genai_amd.utils.tokenizer import embed_tokenizer, llm_tokenizer

    dev = torch.device(args.device)
    torch.manual_seed(0)
    lc = llama_config("llama3-8b")
    hf_cfg = LlamaConfig(vocab_size=lc.vocab_size, hidden_size=lc.hidden, intermediate_size=lc.ffn,
                         num_hidden_layers=args.layers or lc.layers, num_attention_heads=lc.heads,
                         num_key_value_heads=lc.kv_heads, max_position_embeddings=8192,
                         rope_theta=lc.rope_theta, rms_norm_eps=lc.eps, tie_word_embeddings=False,
                         attn_implementation="sdpa", torch_dtype=torch.bfloat16)
    ec = encoder_config("arctic-embed-l")
    bert_cfg = BertConfig(vocab_size=ec.vocab_size, hidden_size=ec.hidden, num_hidden_layers=ec.layers,
                          num_attention_heads=ec.heads, intermediate_size=ec.ffn,
                          max_position_embeddings=512, attn_implementation="sdpa")
    t0 = time.time()
    torch.set_default_dtype(torch.bfloat16)
    with torch.device(dev):
        llm = LlamaForCausalLM(hf_cfg).eval()
        enc = BertModel(bert_cfg, add_pooling_layer=False).eval()
        X = torch.nn.functional.normalize(torch.randn(args.index_size, ec.hidden, dtype=torch.float32), dim=1).bfloat16()
    torch.set_default_dtype(torch.float32)
    print(f"[ref-eq] models + index ready in {time.time() - t0:.1f}s", flush=True)

    tok = llm_tokenizer()
    etok = embed_tokenizer()

    class _Tok:  # RAGPipeline only needs .tok of the LLM and .device of the embedder
        pass

    holder = _Tok()
    holder.tok = tok
    emb_holder = _Tok()
    emb_holder.device = torch.device("cpu")
    docs = SyntheticDocStore(args.index_size)
    rag = RAGPipeline(holder, emb_holder, None, docs, top_k=4)
    gen = TextGen(seed=100)
    prefix = ec.query_prefix

    @torch.inference_mode()
    def serve(questions):
        ids = etok.encode_batch([prefix + q for q in questions])
        L = max(len(x) for x in ids)
        inp = torch.zeros(len(ids), L, dtype=torch.long)
        am = torch.zeros(len(ids), L, dtype=torch.long)
        for i, x in enumerate(ids):
            inp[i, :len(x)] = torch.tensor(x)
            am[i, :len(x)] = 1
        h = enc(input_ids=inp.to(dev), attention_mask=am.to(dev)).last_hidden_state[:, 0]
        q = torch.nn.functional.normalize(h.float(), dim=1).bfloat16()
        sc, ix = torch.topk((q @ X.t()).float(), 4, dim=1)
        sc, ix = sc.tolist(), ix.tolist()
        prompts = [rag.build_prompt(qq, ix[i], sc[i])[0] for i, qq in enumerate(questions)]
        P = max(len(p) for p in prompts)
        pin = torch.zeros(len(prompts), P, dtype=torch.long)
        pam = torch.zeros(len(prompts), P, dtype=torch.long)
        for i, p in enumerate(prompts):   # left padding for batched generate
            pin[i, P - len(p):] = torch.tensor(p)
            pam[i, P - len(p):] = 1
        out = llm.generate(input_ids=pin.to(dev), attention_mask=pam.to(dev), do_sample=True,
                           temperature=0.2, top_p=0.7, top_k=0, max_new_tokens=args.max_tokens,
                           min_new_tokens=args.max_tokens, pad_token_id=0, eos_token_id=None)
        return out, sum(len(p) for p in prompts) / len(prompts)

    # warm-up (kernel selection, allocator)
    serve([gen.question() for _ in range(4)])
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    sync()
    results = []
    for B in [int(b) for b in args.batches.split(",") if b]:
        qs = [gen.question() for _ in range(B)]
        sync()
        t = time.perf_counter()
        out, mean_p = serve(qs)
        sync()
        dt = time.perf_counter() - t
        r = {"stack": "hf-transformers eager + torch brute-force search", "batch": B,
             "qps": round(B / dt, 3), "batch_latency_s": round(dt, 2),
             "mean_prompt_tokens": round(mean_p, 1), "max_tokens": args.max_tokens,
             "output_tokens_per_s": round(B * args.max_tokens / dt, 1),
             "layers": hf_cfg.num_hidden_layers, "index_size": args.index_size}
        print(json.dumps(r), flush=True)
        results.append(r)
        del out
        if dev.type == "cuda":
            torch.cuda.empty_cache()
    best = max(results, key=lambda r: r["qps"])
    summary = {"metric": "end-to-end RAG QPS (reference-equivalent stack)", "best_qps": best["qps"],
               "best_batch": best["batch"], "p50_latency_ms_at_best": round(1000 * best["batch_latency_s"], 1),
               "runs": results}
    print(json.dumps(summary), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(json.dumps(summary) + "\n")


if __name__ == "__main__":
    main()
