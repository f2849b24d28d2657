"""Vision-language serving rate (the NeVA / DePlot image calls of the reference's multimodal
ingest, examples/multimodal_rag/vectorstore/custom_pdf_parser.py:43-71): N concurrent
"Describe this image in detail" requests with distinct synthetic images through
``VisionLanguageModel`` — CLIP tower + projector per image, then continuous-batched prefill
(576 image tokens at 336 px) and decode. Prints one JSON line."""
import argparse
import io
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def png(seed: int, w: int = 640, h: int = 480) -> bytes:
    from PIL import Image

    g = torch.Generator().manual_seed(seed)
    arr = (torch.rand(h // 8, w // 8, 3, generator=g) * 255).to(torch.uint8)
    arr = arr.repeat_interleave(8, 0).repeat_interleave(8, 1).numpy()
    buf = io.BytesIO()
    Image.fromarray(arr).save(buf, format="PNG")
    return buf.getvalue()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llava-1.5-7b")
    ap.add_argument("--images", type=int, default=128)
    ap.add_argument("--max-tokens", type=int, default=128)
    ap.add_argument("--concurrency", type=int, default=64)
    ap.add_argument("--encode-batch", type=int, default=32, help="images per batched tower pass")
    args = ap.parse_args()
    from nv_genai_amd.engine.llm_engine import EngineConfig, SamplingParams
    from nv_genai_amd.models.vision import VisionLanguageModel, vlm_config

    cfg = vlm_config(args.model)
    vlm = VisionLanguageModel(cfg, engine_cfg=EngineConfig(model=cfg.llm, max_num_seqs=args.concurrency,
                                                          max_model_len=4096, max_batched_tokens=16384))
    imgs = [png(i) for i in range(args.images)]
    p = SamplingParams(temperature=0.2, top_p=0.7, max_tokens=args.max_tokens, ignore_eos=True)

    def msgs(i):
        return [{"role": "user", "content": [{"type": "text", "text": "Describe this image in detail"},
                                             {"type": "image", "image": imgs[i]}]}]

    vlm.generate([msgs(i) for i in range(min(8, args.images))], p)     # warm-up (graphs, allocator)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pending, nxt, done, enc_s = [], 0, [], 0.0
    feats = {}
    while nxt < args.images or pending:
        while nxt < args.images and len(pending) < args.concurrency:
            te = time.perf_counter()
            if imgs[nxt] not in feats:
                # the next chunk of arriving images goes through the tower as one batch
                # (host preprocessing on threads), inside the timed region
                feats.update(vlm.image_features(imgs[nxt:nxt + args.encode_batch]))
            pending.append(vlm.submit(msgs(nxt), p, features=feats))
            enc_s += time.perf_counter() - te
            nxt += 1
        vlm.engine.step()
        still = []
        for r in pending:
            (done if r.finished else still).append(r)
        pending = still
    vlm.engine.run_until_done()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    lat = sorted(r.latency for r in done)
    print(json.dumps({"metric": "VLM describe rate", "model": args.model, "images": args.images,
                      "images_per_s": round(args.images / dt, 2),
                      "output_tokens_per_s": round(args.images * args.max_tokens / dt, 1),
                      "p50_latency_s": round(lat[len(lat) // 2], 3), "image_tokens": cfg.vision.num_patches,
                      "host_encode_submit_s": round(enc_s, 2), "wall_s": round(dt, 2)}), flush=True)


if __name__ == "__main__":
    main()
