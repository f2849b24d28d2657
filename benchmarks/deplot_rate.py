"""DePlot chart-to-table rate (the reference's ``process_graph`` call of its multimodal ingest,
examples/multimodal_rag/vectorstore/custom_pdf_parser.py:55-71; BASELINE.json configs[4]):
synthetic bar-chart PNGs -> VQA header render + Pix2Struct patches (host) -> batched encoder
(packed varlen MFMA attention) -> hipGraph greedy decode of ``--max-tokens`` table tokens.
Random-init weights of the DePlot (pix2struct-base) architecture; EOS is ignored so every
image decodes the same number of tokens. Prints one JSON line."""
import argparse
import io
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def chart_png(seed: int, w: int = 640, h: int = 480) -> bytes:
    """A bar chart with axes, bars and labels (text-and-shape structure like a real chart)."""
    import random

    from PIL import Image, ImageDraw

    rng = random.Random(seed)
    im = Image.new("RGB", (w, h), "white")
    d = ImageDraw.Draw(im)
    d.line([(60, 20), (60, h - 40), (w - 20, h - 40)], fill="black", width=2)
    n = rng.randint(3, 9)
    bw = (w - 100) // n
    for i in range(n):
        v = rng.randint(20, h - 80)
        x0 = 70 + i * bw
        d.rectangle([x0, h - 40 - v, x0 + bw - 12, h - 41], fill=(rng.randint(0, 200), rng.randint(0, 200), 220))
        d.text((x0, h - 32), f"c{i}", fill="black")
        d.text((x0, h - 55 - v), str(v), fill="black")
    d.text((w // 2 - 40, 4), f"chart {seed}", fill="black")
    buf = io.BytesIO()
    im.save(buf, format="PNG")
    return buf.getvalue()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="deplot")
    ap.add_argument("--images", type=int, default=128)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--max-tokens", type=int, default=128)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--host-threads", type=int, default=8)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from nv_genai_amd.models.pix2struct import DePlot

    dp = DePlot(args.model)
    dev = dp.model.device
    imgs = [chart_png(i) for i in range(args.images)]
    # warm-up batch (kernels, hipBLASLt handles, graph pool)
    dp.model.generate([dp.patches(im) for im in imgs[: args.batch]], max_new_tokens=args.max_tokens,
                      use_graph=False if args.no_graph else None, ignore_eos=True)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    from concurrent.futures import ThreadPoolExecutor

    from nv_genai_amd.models.pix2struct import flatten_patches, render_header

    cfg = dp.cfg

    workers = ThreadPoolExecutor(args.host_threads)

    def host(batch):
        """PNG decode + VQA header render (PIL, host; PIL drops the GIL) for one batch, fanned
        out over worker threads while the GPU decodes the previous batch."""
        if not cfg.is_vqa:
            return list(batch)
        return list(workers.map(lambda im: render_header(im, dp.PROMPT), batch))

    t_pre = t_enc = t_gen = 0.0
    t0 = time.perf_counter()
    toks = 0
    batches = [imgs[s:s + args.batch] for s in range(0, args.images, args.batch)]
    with ThreadPoolExecutor(1) as pool:
        fut = pool.submit(host, batches[0])
        for i in range(len(batches)):
            a = time.perf_counter()
            arrs = fut.result()
            if i + 1 < len(batches):
                fut = pool.submit(host, batches[i + 1])
            ps = [flatten_patches(x, cfg.max_patches, cfg.patch, device=dev) for x in arrs]
            b = time.perf_counter()
            out = dp.model.generate(ps, max_new_tokens=args.max_tokens,
                                    use_graph=False if args.no_graph else None, ignore_eos=True)
            if dev.type == "cuda":
                torch.cuda.synchronize()
            c = time.perf_counter()
            t_pre += b - a
            t_gen += c - b
            toks += sum(len(o) for o in out)
    wall = time.perf_counter() - t0
    workers.shutdown()
    # encoder-only time of one batch (the rest of generate is decode)
    ps = [dp.patches(im) for im in imgs[: args.batch]]
    if dev.type == "cuda":
        torch.cuda.synchronize()
    e0 = time.perf_counter()
    dp.model.encode(ps)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t_enc = time.perf_counter() - e0
    line = {"metric": "DePlot chart-to-table rate", "model": args.model, "images": args.images,
            "batch": args.batch, "max_tokens": args.max_tokens, "graph": not args.no_graph,
            "patches_per_image": int(ps[0].shape[0]), "images_per_s": round(args.images / wall, 2),
            "output_tok_per_s": round(toks / wall, 1), "wall_s": round(wall, 3),
            "host_preprocess_wait_s": round(t_pre, 3), "generate_s": round(t_gen, 3),
            "encoder_ms_per_batch": round(1e3 * t_enc, 2),
            "data": "synthetic bar charts; random-init weights of the architecture",
            "dtype": str(dp.model.dtype).replace("torch.", "")}
    s = json.dumps(line)
    print(s, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
