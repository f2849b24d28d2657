"""Supervised fine-tuning (full or LoRA) of the Llama family, data-parallel over RCCL
(reference: models/Gemma/{lora,sft}.ipynb, models/StarCoder2,
models/Codegemma — NeMo ``megatron_gpt_finetuning`` with ``micro_batch_size``,
``global_batch_size``, ``max_steps``, ``val_check_interval``, ``peft_scheme``, bf16).

* data: JSONL with ``input``/``output`` (NeMo SFT format) or ``prompt``/``completion``; the
  loss covers the output tokens only (``answer_only_loss``), sequences are right padded per
  micro-batch and truncated to ``max_seq_len``;
* optimisation: AdamW on fp32 masters (full) or fp32 adapters (LoRA), cosine schedule with
  linear warm-up, global-norm clipping, gradient accumulation to ``global_batch``;
* parallelism: one process per GPU; gradients bucketed and all-reduced during backward
  (``parallel/grad_sync.py``); each rank reads a disjoint strided shard of every global batch;
* checkpoint/resume: trainable tensors (safetensors), optimizer state, step, RNG states and
  the data cursor, written atomically every ``save_every`` steps; ``resume`` restores all of it
  so a resumed run is step-for-step identical to an uninterrupted one.

``python -m nv_genai_amd.training.sft --model llama-tiny --data train.jsonl --lora``
"""
from __future__ import annotations

import argparse
import json
import math
import os
import random
import shutil
import time
from dataclasses import asdict, dataclass
from typing import Dict, List, Optional, Sequence

import torch

from . import functional as Fn
from .lora import LoRA, LoRAConfig


@dataclass
class TrainConfig:
    lr: float = 1e-4
    min_lr: float = 0.0
    weight_decay: float = 0.01
    betas: tuple = (0.9, 0.98)
    warmup_steps: int = 10
    max_steps: int = 100
    micro_batch: int = 1
    global_batch: int = 8
    max_seq_len: int = 2048
    grad_clip: float = 1.0
    grad_ckpt: bool = False
    seed: int = 1234
    save_every: int = 0
    log_every: int = 10
    bucket_mb: float = 256.0


def load_jsonl(path: str) -> List[dict]:
    with open(path) as f:
        return [json.loads(ln) for ln in f if ln.strip()]


def encode_example(tok, ex: dict, max_len: int, bos: Optional[int] = None, eos: Optional[int] = None):
    """→ (ids, labels) with labels = next token on output positions, -100 elsewhere."""
    src = ex.get("input", ex.get("prompt", ""))
    tgt = ex.get("output", ex.get("completion", ""))
    p = ([bos] if bos is not None else []) + tok.encode(src)
    a = tok.encode(tgt) + ([eos] if eos is not None else [])
    ids = (p + a)[: max_len + 1]
    labels = [-100] * (len(p) - 1) + a
    labels = labels[: len(ids) - 1]
    return ids[:-1], labels


def collate(batch, pad_id: int = 0):
    S = max(len(i) for i, _ in batch)
    ids = torch.full((len(batch), S), pad_id, dtype=torch.long)
    lab = torch.full((len(batch), S), -100, dtype=torch.long)
    for b, (i, y) in enumerate(batch):
        ids[b, : len(i)] = torch.tensor(i)
        lab[b, : len(y)] = torch.tensor(y)
    return ids, lab


def lr_at(step: int, cfg: TrainConfig) -> float:
    if step < cfg.warmup_steps:
        return cfg.lr * (step + 1) / cfg.warmup_steps
    t = (step - cfg.warmup_steps) / max(1, cfg.max_steps - cfg.warmup_steps)
    return cfg.min_lr + 0.5 * (cfg.lr - cfg.min_lr) * (1 + math.cos(math.pi * min(1.0, t)))


class Trainer:
    """Generic loop: ``loss_fn(micro_batch) -> scalar``, trainable tensors ``named``."""

    def __init__(self, named: Dict[str, torch.Tensor], loss_fn, batches: Sequence, cfg: TrainConfig,
                 group=None, ckpt_dir: Optional[str] = None, on_save=None, fused: bool = False):
        import torch.distributed as dist

        from ..parallel.grad_sync import GradBucketer, broadcast_params

        self.named, self.loss_fn, self.data, self.cfg = named, loss_fn, list(batches), cfg
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.params = list(named.values())
        broadcast_params(self.params, group=group)
        self.sync = GradBucketer(self.params, group=group, bucket_mb=cfg.bucket_mb)
        decay = [p for n, p in named.items() if p.ndim >= 2]
        nodecay = [p for n, p in named.items() if p.ndim < 2]
        self.opt = torch.optim.AdamW([{"params": decay, "weight_decay": cfg.weight_decay},
                                      {"params": nodecay, "weight_decay": 0.0}], lr=cfg.lr, betas=cfg.betas,
                                     **({"fused": True} if fused else {}))
        self.step = 0
        self.cursor = 0
        self.ckpt_dir = ckpt_dir
        self.on_save = on_save
        self.history: List[float] = []
        self.accum = max(1, cfg.global_batch // (cfg.micro_batch * self.world))
        self.group = group

    # -------------------------------------------------------------- data
    def _next_micro_batches(self) -> List:
        """The micro-batches this rank runs for one optimizer step (strided shard of a
        global batch; the cursor wraps around the epoch)."""
        out = []
        per_step = self.accum * self.world
        for a in range(self.accum):
            j = (self.cursor + a * self.world + self.rank) % len(self.data)
            out.append(self.data[j])
        self.cursor = (self.cursor + per_step) % len(self.data)
        return out

    # -------------------------------------------------------------- step
    def train_step(self) -> float:
        import torch.distributed as dist

        cfg = self.cfg
        for g in self.opt.param_groups:
            g["lr"] = lr_at(self.step, cfg)
        self.opt.zero_grad(set_to_none=True)
        mbs = self._next_micro_batches()
        total = 0.0
        for i, mb in enumerate(mbs):
            self.sync.sync(i == len(mbs) - 1)
            loss = self.loss_fn(mb) / len(mbs)
            loss.backward()
            total += float(loss.detach())
        self.sync.finish()
        if cfg.grad_clip:
            torch.nn.utils.clip_grad_norm_(self.params, cfg.grad_clip)
        self.opt.step()
        self.step += 1
        if self.world > 1:
            t = torch.tensor([total], dtype=torch.float64, device=self.params[0].device)
            dist.all_reduce(t, group=self.group)
            total = float(t) / self.world
        self.history.append(total)
        if self.ckpt_dir and cfg.save_every and self.step % cfg.save_every == 0:
            self.save(self.ckpt_dir)
        return total

    def fit(self, steps: Optional[int] = None, log=print) -> List[float]:
        n = steps if steps is not None else self.cfg.max_steps - self.step
        t0 = time.perf_counter()
        for _ in range(n):
            loss = self.train_step()
            if self.rank == 0 and self.cfg.log_every and self.step % self.cfg.log_every == 0:
                log(f"step {self.step} loss {loss:.4f} lr {lr_at(self.step - 1, self.cfg):.2e} "
                    f"{(time.perf_counter() - t0) / max(1, self.step):.3f}s/step")
        return self.history

    # -------------------------------------------------------------- checkpoint
    def state(self) -> dict:
        return {"step": self.step, "cursor": self.cursor, "history": self.history,
                "cfg": {k: list(v) if isinstance(v, tuple) else v for k, v in asdict(self.cfg).items()}}

    def save(self, path: str) -> None:
        """Atomic: written to ``path.tmp`` then renamed. Only rank 0 writes (the
        trainable state is replicated)."""
        if self.rank != 0:
            return
        from safetensors.torch import save_file

        tmp = path.rstrip("/") + ".tmp"
        shutil.rmtree(tmp, ignore_errors=True)
        os.makedirs(tmp)
        save_file({n: p.detach().cpu().contiguous() for n, p in self.named.items()},
                  os.path.join(tmp, "trainable.safetensors"))
        torch.save({"opt": self.opt.state_dict(), "cpu_rng": torch.get_rng_state()},
                   os.path.join(tmp, "optim.pt"))
        with open(os.path.join(tmp, "trainer_state.json"), "w") as f:
            json.dump(self.state(), f)
        if self.on_save:
            self.on_save(tmp)
        if os.path.exists(path):
            shutil.rmtree(path)
        os.replace(tmp, path)

    def resume(self, path: str) -> bool:
        if not os.path.exists(os.path.join(path, "trainer_state.json")):
            return False
        from safetensors.torch import load_file

        sd = load_file(os.path.join(path, "trainable.safetensors"))
        with torch.no_grad():
            for n, p in self.named.items():
                p.copy_(sd[n].to(p.device, p.dtype))
        o = torch.load(os.path.join(path, "optim.pt"), weights_only=True, map_location="cpu")
        self.opt.load_state_dict(o["opt"])
        torch.set_rng_state(o["cpu_rng"])
        with open(os.path.join(path, "trainer_state.json")) as f:
            st = json.load(f)
        self.step, self.cursor, self.history = st["step"], st["cursor"], st["history"]
        return True


def sft_trainer(model, tok, examples: Sequence[dict], cfg: TrainConfig, lora: Optional[LoRAConfig] = None,
                group=None, ckpt_dir: Optional[str] = None):
    """Build a Trainer for LoRA (``lora`` given) or full fine-tuning of ``model``.
    Returns (trainer, adapter_or_params)."""
    dev = model.embed.device
    random.seed(cfg.seed)
    torch.manual_seed(cfg.seed)
    enc = [encode_example(tok, ex, cfg.max_seq_len, model.cfg.bos_id, model.cfg.eos_ids[0]) for ex in examples]
    batches = [collate(enc[i:i + cfg.micro_batch]) for i in range(0, len(enc), cfg.micro_batch)]
    if lora is not None:
        ad = LoRA(model, lora, seed=cfg.seed)
        named = dict(ad.named_parameters())

        def loss_fn(mb):
            ids, lab = mb[0].to(dev), mb[1].to(dev)
            with torch.autocast(dev.type, dtype=torch.bfloat16):
                h = Fn.llama_hidden(model, ids, linear=ad.linear, grad_ckpt=cfg.grad_ckpt)
                return Fn.lm_loss(model, h, lab)
        return Trainer(named, loss_fn, batches, cfg, group, ckpt_dir), ad
    params = Fn.trainable_params(model, "llama")
    named = {(k if isinstance(k, str) else f"layers.{k[0]}.{k[1]}"): v for k, v in params.items()}

    def loss_fn(mb):
        ids, lab = mb[0].to(dev), mb[1].to(dev)
        with torch.autocast(dev.type, dtype=torch.bfloat16):
            h = Fn.llama_hidden(model, ids, params=params, grad_ckpt=cfg.grad_ckpt)
            return Fn.lm_loss(model, h, lab, params=params)
    return Trainer(named, loss_fn, batches, cfg, group, ckpt_dir), params


def main(argv=None):
    ap = argparse.ArgumentParser(description="SFT / LoRA fine-tuning (one process per GPU)")
    ap.add_argument("--model", default="llama-tiny")
    ap.add_argument("--weights", default=None, help="directory of HF safetensors")
    ap.add_argument("--data", required=True)
    ap.add_argument("--lora", action="store_true")
    ap.add_argument("--lora-r", type=int, default=32)
    ap.add_argument("--lora-alpha", type=float, default=32.0)
    ap.add_argument("--lora-targets", default="qkv")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--micro-batch", type=int, default=1)
    ap.add_argument("--global-batch", type=int, default=8)
    ap.add_argument("--max-seq-len", type=int, default=2048)
    ap.add_argument("--grad-ckpt", action="store_true")
    ap.add_argument("--ckpt-dir", default=None)
    ap.add_argument("--save-every", type=int, default=0)
    ap.add_argument("--out", default=None, help="write merged HF weights (full) or the adapter (LoRA) here")
    args = ap.parse_args(argv)
    from ..models.config import llama_config
    from ..models.llama import LlamaModel
    from ..parallel.dist import init_distributed
    from ..utils.tokenizer import llm_tokenizer

    pctx = init_distributed()
    dev = pctx.device if pctx.device.type == "cuda" else torch.device("cuda" if torch.cuda.is_available() else "cpu")
    weights = None
    if args.weights:
        from ..utils.checkpoint import load_weights

        weights = load_weights(args.weights)
    model = LlamaModel(llama_config(args.model), dev, weights=weights)
    cfg = TrainConfig(lr=args.lr, max_steps=args.steps, micro_batch=args.micro_batch, global_batch=args.global_batch,
                      max_seq_len=args.max_seq_len, grad_ckpt=args.grad_ckpt, save_every=args.save_every)
    lcfg = LoRAConfig(r=args.lora_r, alpha=args.lora_alpha, targets=tuple(args.lora_targets.split(","))) \
        if args.lora else None
    tr, state = sft_trainer(model, llm_tokenizer(), load_jsonl(args.data), cfg, lcfg, ckpt_dir=args.ckpt_dir)
    if args.ckpt_dir and tr.resume(args.ckpt_dir):
        print(f"resumed at step {tr.step}")
    tr.fit(args.steps - tr.step)
    if args.out and tr.rank == 0:
        if args.lora:
            state.save(args.out)
        else:
            from safetensors.torch import save_file

            Fn.write_back(model, state, "llama")
            os.makedirs(args.out, exist_ok=True)
            save_file({k: v.cpu().contiguous() for k, v in model.state_dict().items()},
                      os.path.join(args.out, "model.safetensors"))


if __name__ == "__main__":
    main()
