"""Small-language-model pretraining from scratch, then SFT (reference:
models/NeMo/slm/slm_pretraining_sft.ipynb#cell 18 — a 12-layer / 768-hidden GPT pretrained with
NeMo ``megatron_gpt_pretraining`` (packed ``seq_length`` samples from a tokenised corpus,
``fused_adam``, cosine LR with warm-up, ``micro_batch_size`` / ``global_batch_size``), then
fine-tuned with ``megatron_gpt_finetuning``).

The model is this framework's Llama architecture at SLM scale (``slm-125m``: 12 layers, hidden
768, 12 heads, SwiGLU 2048, RoPE), so a pretrained checkpoint is served by the same engine and
HIP kernels as Llama-3 and fine-tuned by :mod:`.sft`.

* data: text files / JSONL ``{"text": ...}`` tokenised, each document terminated by EOS,
  concatenated and cut into ``seq_len + 1``-token windows (the NeMo "packed" layout): every
  token is a training target, no padding;
* optimisation: :class:`.sft.Trainer` — AdamW (the fused multi-tensor kernel on GPU, the
  ``fused_adam`` of the notebook), cosine schedule, clipping, gradient accumulation, bucketed
  DP all-reduce overlapped with backward, atomic checkpoint / exact resume.

``torchrun --nproc-per-node 8 -m nv_genai_amd.training.pretrain --data corpus.jsonl --out slm/``
"""
from __future__ import annotations

import argparse
import json
import os
from typing import Iterable, List, Optional, Sequence

import torch

from . import functional as Fn
from .sft import TrainConfig, Trainer


def iter_texts(paths: Sequence[str]) -> Iterable[str]:
    for p in paths:
        with open(p) as f:
            if p.endswith(".jsonl"):
                for ln in f:
                    if ln.strip():
                        yield json.loads(ln).get("text", "")
            else:
                yield f.read()


def pack(token_docs: Iterable[List[int]], seq_len: int, eos: int) -> torch.Tensor:
    """Concatenate documents (each + EOS) and cut into ``[N, seq_len + 1]`` windows; the
    ragged tail is dropped (NeMo's packed-dataset behaviour)."""
    stream: List[int] = []
    for d in token_docs:
        stream.extend(d)
        stream.append(eos)
    n = len(stream) // (seq_len + 1)
    if n == 0:
        raise ValueError(f"corpus of {len(stream)} tokens is shorter than one {seq_len + 1}-token window")
    return torch.tensor(stream[: n * (seq_len + 1)], dtype=torch.long).view(n, seq_len + 1)


def init_slm(model, seed: int = 1234, std: float = 0.02) -> None:
    """GPT-style init for training from scratch: N(0, std) projections, the residual
    output projections (O, down) scaled by 1/sqrt(2·layers), unit norms."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    out_std = std / (2 * len(model.layers)) ** 0.5
    with torch.no_grad():
        def fill(t, s):
            t.copy_((torch.randn(t.shape, generator=g) * s).to(t.dtype))
        fill(model.embed, std)
        fill(model.lm_head, std)
        for L in model.layers:
            fill(L["wqkv"], std)
            fill(L["wgu"], std)
            fill(L["wo"], out_std)
            fill(L["wd"], out_std)
            L["attn_norm"].fill_(1.0)
            L["mlp_norm"].fill_(1.0)
        model.final_norm.fill_(1.0)


def pretrain_trainer(model, windows: torch.Tensor, cfg: TrainConfig, group=None,
                     ckpt_dir: Optional[str] = None):
    """Full-parameter LM pretraining on packed windows. Returns (trainer, fp32 params)."""
    dev = model.embed.device
    torch.manual_seed(cfg.seed)
    batches = [(windows[i:i + cfg.micro_batch, :-1], windows[i:i + cfg.micro_batch, 1:])
               for i in range(0, windows.shape[0] - cfg.micro_batch + 1, cfg.micro_batch)]
    params = Fn.trainable_params(model, "llama")
    named = {(k if isinstance(k, str) else f"layers.{k[0]}.{k[1]}"): v for k, v in params.items()}

    def loss_fn(mb):
        ids, lab = mb[0].to(dev), mb[1].to(dev)
        with torch.autocast(dev.type, dtype=torch.bfloat16):
            h = Fn.llama_hidden(model, ids, params=params, grad_ckpt=cfg.grad_ckpt)
            return Fn.lm_loss(model, h, lab, params=params)
    return Trainer(named, loss_fn, batches, cfg, group, ckpt_dir, fused=dev.type == "cuda"), params


def main(argv=None):
    ap = argparse.ArgumentParser(description="SLM pretraining (one process per GPU)")
    ap.add_argument("--model", default="slm-125m")
    ap.add_argument("--data", nargs="+", required=True, help="text files or JSONL with a 'text' field")
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--lr", type=float, default=6e-4)
    ap.add_argument("--min-lr", type=float, default=6e-5)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--micro-batch", type=int, default=8)
    ap.add_argument("--global-batch", type=int, default=64)
    ap.add_argument("--grad-ckpt", action="store_true")
    ap.add_argument("--ckpt-dir", default=None)
    ap.add_argument("--save-every", type=int, default=0)
    ap.add_argument("--out", default=None, help="write the pretrained weights (safetensors) here")
    args = ap.parse_args(argv)
    from ..models.config import llama_config
    from ..models.llama import LlamaModel
    from ..parallel.dist import init_distributed
    from ..utils.tokenizer import llm_tokenizer

    pctx = init_distributed()
    dev = pctx.device if pctx.device.type == "cuda" else torch.device("cuda" if torch.cuda.is_available() else "cpu")
    mcfg = llama_config(args.model)
    model = LlamaModel(mcfg, dev)
    init_slm(model)
    tok = llm_tokenizer()
    windows = pack((tok.encode(t) for t in iter_texts(args.data)), args.seq_len, mcfg.eos_ids[0])
    cfg = TrainConfig(lr=args.lr, min_lr=args.min_lr, warmup_steps=args.warmup, max_steps=args.steps,
                      micro_batch=args.micro_batch, global_batch=args.global_batch,
                      max_seq_len=args.seq_len, grad_ckpt=args.grad_ckpt, save_every=args.save_every,
                      betas=(0.9, 0.95), weight_decay=0.1)
    tr, params = pretrain_trainer(model, windows, cfg, ckpt_dir=args.ckpt_dir)
    if args.ckpt_dir and tr.resume(args.ckpt_dir):
        print(f"resumed at step {tr.step}")
    tr.fit(args.steps - tr.step)
    if args.out and tr.rank == 0:
        from safetensors.torch import save_file

        Fn.write_back(model, params, "llama")
        os.makedirs(args.out, exist_ok=True)
        save_file({k: v.cpu().contiguous() for k, v in model.state_dict().items()},
                  os.path.join(args.out, "model.safetensors"))


if __name__ == "__main__":
    main()
