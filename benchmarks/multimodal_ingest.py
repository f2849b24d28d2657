"""Multimodal RAG ingestion on one MI355X (BASELINE.json configs[4]: Llama-3-8B + DePlot +
NeVA-22B image/table ingestion). The reference's per-image path
(examples/multimodal_rag/vectorstore/custom_pdf_parser.py:43-71, ``is_graph`` ->
``process_graph``; chains.py of our example mirrors it) is run for a batch of chart images,
with every engine in this process on the same GPU:

1. NeVA-22B "Describe this image in detail" (LLaVA-architecture VLM: CLIP tower + projector,
   continuous-batched 22B decoder);
2. DePlot "Generate underlying data table of the figure below:" (Pix2Struct encoder-decoder,
   hipGraph decode);
3. Llama-3-8B "Explain the following linearized table." with the reference's chart system
   prompt (continuous batching);
4. arctic-embed-l embedding of description + explanation and insertion into the in-HBM index.

Every image is a chart (the workload: a chart-heavy deck), so step 1's "is it a graph?" branch
is taken for all of them — with random-init weights the description text cannot decide it.
DePlot (steps 1 and 2 are independent) runs concurrently with the NeVA pass on a side stream
(``--overlap 0``: one after the other); the explain and embed stages follow. The JSON line has
the end-to-end images/s and each stage's time. Synthetic charts, random-init weights of each
architecture, EOS ignored (fixed token counts)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from benchmarks.deplot_rate import chart_png  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=64)
    ap.add_argument("--vlm", default="neva-22b")
    ap.add_argument("--deplot", default="deplot")
    ap.add_argument("--llm", default="llama3-8b")
    ap.add_argument("--embed", default="arctic-embed-l")
    ap.add_argument("--describe-tokens", type=int, default=128)
    ap.add_argument("--table-tokens", type=int, default=128)
    ap.add_argument("--explain-tokens", type=int, default=256)
    ap.add_argument("--deplot-batch", type=int, default=32)
    ap.add_argument("--overlap", type=int, default=1,
                    help="run DePlot concurrently with the NeVA pass (side stream + worker thread)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from nv_genai_amd.engine.embed_engine import EmbeddingEngine
    from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine, SamplingParams
    from nv_genai_amd.examples.multimodal_rag.chains import CHART_SYSTEM
    from nv_genai_amd.index.flat import FlatIndex
    from nv_genai_amd.models.pix2struct import DePlot
    from nv_genai_amd.models.vision import VisionLanguageModel, vlm_config

    t_setup = time.perf_counter()
    N = args.images
    vc = vlm_config(args.vlm)
    vlm = VisionLanguageModel(vc, engine_cfg=EngineConfig(model=vc.llm, max_num_seqs=max(N, 8), max_model_len=4096,
                                                          max_batched_tokens=16384, kv_cache_fraction=0.25))
    llm = LLMEngine(EngineConfig(model=args.llm, max_num_seqs=max(N, 8), max_model_len=4096,
                                 max_batched_tokens=16384, kv_cache_fraction=0.25))
    dp = DePlot(args.deplot)
    emb = EmbeddingEngine(args.embed)
    index = FlatIndex(emb.dim, "cosine", "cuda" if torch.cuda.is_available() else "cpu", capacity=4 * N)
    imgs = [chart_png(i) for i in range(N)]
    p_desc = SamplingParams(temperature=0.2, top_p=0.7, max_tokens=args.describe_tokens, ignore_eos=True)
    p_expl = SamplingParams(temperature=0.2, top_p=0.7, max_tokens=args.explain_tokens, ignore_eos=True)
    describe = "Describe this image in detail [labels: creativity:0,quality:9,complexity:0,verbosity:9]"

    def vlm_msgs(im):
        return [{"role": "user", "content": [{"type": "text", "text": describe}, {"type": "image", "image": im}]}]

    # warm-up of every engine (graphs, allocator pools, hipBLASLt handles)
    vlm.generate([vlm_msgs(im) for im in imgs[:4]], p_desc)
    dp.describe_batch(imgs[:4], max_new_tokens=8)
    llm.generate([llm.apply_chat_template([{"role": "user", "content": "warm up"}])] * 4, p_expl)
    emb.embed(["warm up"] * 4)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    setup_s = time.perf_counter() - t_setup

    st = {}
    t0 = time.perf_counter()

    def deplot_tables():
        a = time.perf_counter()
        out = [dp.tok.decode(o) for o in dp.generate_many(imgs, batch=args.deplot_batch,
                                                          max_new_tokens=args.table_tokens, ignore_eos=True)]
        st["deplot_table_s"] = time.perf_counter() - a
        return out

    if args.overlap and torch.cuda.is_available():
        # DePlot (latency-bound small decode kernels, its own hipGraph) on a side stream in a
        # worker thread, while the VLM engine steps on the main thread's stream
        from concurrent.futures import ThreadPoolExecutor

        side = torch.cuda.Stream()

        def on_side():
            with torch.cuda.stream(side):
                out = deplot_tables()
            side.synchronize()
            return out

        with ThreadPoolExecutor(1) as ex:
            fut = ex.submit(on_side)
            a = time.perf_counter()
            descs = [r.text for r in vlm.generate([vlm_msgs(im) for im in imgs], p_desc)]
            st["neva_describe_s"] = time.perf_counter() - a
            tables = fut.result()
    else:
        a = time.perf_counter()
        descs = [r.text for r in vlm.generate([vlm_msgs(im) for im in imgs], p_desc)]
        st["neva_describe_s"] = time.perf_counter() - a
        tables = deplot_tables()
    st["describe_and_table_s"] = time.perf_counter() - t0
    a = time.perf_counter()
    prompts = [llm.apply_chat_template([{"role": "system", "content": CHART_SYSTEM},
                                        {"role": "user", "content": "Explain the following linearized table. " + t}])
               for t in tables]
    expl = [r.text for r in llm.generate(prompts, p_expl)]
    st["llm_explain_s"] = time.perf_counter() - a
    a = time.perf_counter()
    vecs = emb.embed([d + "\n" + e for d, e in zip(descs, expl)], input_type="passage")
    index.add(vecs)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    st["embed_index_s"] = time.perf_counter() - a
    wall = time.perf_counter() - t0
    line = {"metric": "multimodal ingestion rate (NeVA describe -> DePlot table -> LLM explain -> embed + index)",
            "value": round(N / wall, 3), "unit": "images/s", "images": N, "wall_s": round(wall, 2),
            **{k: round(v, 2) for k, v in st.items()},
            "overlap": bool(args.overlap),
            "models": {"vlm": args.vlm, "deplot": args.deplot, "llm": args.llm, "embed": args.embed},
            "tokens": {"describe": args.describe_tokens, "table": args.table_tokens, "explain": args.explain_tokens},
            "mean_explain_prompt_tokens": round(sum(map(len, prompts)) / N, 1),
            "index_size": index.size if hasattr(index, "size") else N, "setup_s": round(setup_s, 1),
            "n_gpus": 1, "dtype": "bf16",
            "data": "synthetic bar charts; random-init weights of each architecture; every image taken as a chart"}
    s = json.dumps(line)
    print(s, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
