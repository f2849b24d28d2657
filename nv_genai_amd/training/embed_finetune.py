"""Contrastive fine-tuning of the embedding encoder (reference:
retriever_customization.ipynb#cell 29 — NeMo ``megatron_sbert_finetune.py`` with
``global_batch_size=8``, ``micro_batch_size=4``, ``hard_negatives_to_train=4``, 1 epoch).

Loss (SBERT multiple-negatives ranking): for a micro-batch of B queries, each with one
positive and ``hard_negatives`` mined negatives, the candidate set is all B·(1+h) passages
of the batch; logits = scale · cos(q, p) and the target of query i is its own positive, so
every other query's positive and negatives act as in-batch negatives. Queries get the
model's query prefix, passages its passage prefix (asymmetric embedding). Encoder weights
train as fp32 masters under bf16 autocast; data parallelism, bucketed gradient all-reduce and
checkpoint/resume come from the shared ``Trainer``.

``python -m nv_genai_amd.training.embed_finetune --model encoder-tiny --data train.json``
(``data``: the JSON list written by ``hard_negatives.build_training_records``).
"""
from __future__ import annotations

import argparse
import json
import os
import random
from typing import List, Optional, Sequence

import torch
import torch.nn.functional as F

from . import functional as Fn
from .sft import TrainConfig, Trainer


def _pad(seqs: Sequence[Sequence[int]]):
    S = max(len(s) for s in seqs)
    ids = torch.zeros(len(seqs), S, dtype=torch.long)
    mask = torch.zeros(len(seqs), S, dtype=torch.long)
    for i, s in enumerate(seqs):
        ids[i, : len(s)] = torch.tensor(s)
        mask[i, : len(s)] = 1
    return ids, mask


def make_batches(engine, records: Sequence[dict], micro_batch: int, hard_negatives: int = 4,
                 max_len: int = 512, seed: int = 0):
    """Tokenised micro-batches: (q_ids, q_mask, p_ids, p_mask) with passages laid out as
    [pos_0, negs_0..., pos_1, negs_1...]. Records with too few negatives are padded by
    sampling other records' positives."""
    rng = random.Random(seed)
    all_pos = [r["pos_doc"][0] for r in records]
    out = []
    for s in range(0, len(records), micro_batch):
        chunk = records[s:s + micro_batch]
        qs = engine.tokenize([r["question"] for r in chunk], "query")
        ps: List[str] = []
        for r in chunk:
            negs = list(r.get("neg_doc", []))[:hard_negatives]
            while len(negs) < hard_negatives:
                cand = rng.choice(all_pos)
                if cand != r["pos_doc"][0]:
                    negs.append(cand)
            ps += [r["pos_doc"][0]] + negs
        pt = engine.tokenize(ps, "passage")
        qs = [q[:max_len] for q in qs]
        pt = [p[:max_len] for p in pt]
        out.append((*_pad(qs), *_pad(pt)))
    return out


def contrastive_loss(q: torch.Tensor, p: torch.Tensor, group: int, scale: float = 20.0) -> torch.Tensor:
    """q [B, H], p [B·group, H] unit vectors; the positive of query i is p[i·group]."""
    logits = scale * (q @ p.t())
    target = torch.arange(q.shape[0], device=q.device) * group
    return F.cross_entropy(logits.float(), target)


def embed_trainer(engine, records: Sequence[dict], cfg: TrainConfig, hard_negatives: int = 4,
                  scale: float = 20.0, group=None, ckpt_dir: Optional[str] = None):
    model = engine.model
    dev = engine.device
    torch.manual_seed(cfg.seed)
    params = Fn.trainable_params(model, "encoder")
    named = {(k if isinstance(k, str) else f"layers.{k[0]}.{k[1]}"): v for k, v in params.items()}
    batches = make_batches(engine, records, cfg.micro_batch, hard_negatives, cfg.max_seq_len, cfg.seed)

    def loss_fn(mb):
        qi, qm, pi, pm = (t.to(dev) for t in mb)
        with torch.autocast(dev.type, dtype=torch.bfloat16):
            q = Fn.encoder_embed(model, qi, qm, params, cfg.grad_ckpt)
            p = Fn.encoder_embed(model, pi, pm, params, cfg.grad_ckpt)
        return contrastive_loss(q, p, 1 + hard_negatives, scale)

    return Trainer(named, loss_fn, batches, cfg, group, ckpt_dir), params


def main(argv=None):
    ap = argparse.ArgumentParser(description="Contrastive fine-tuning of the embedding encoder")
    ap.add_argument("--model", default="encoder-tiny")
    ap.add_argument("--data", required=True)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--lr", type=float, default=5e-6)
    ap.add_argument("--micro-batch", type=int, default=4)
    ap.add_argument("--global-batch", type=int, default=8)
    ap.add_argument("--hard-negatives", type=int, default=4)
    ap.add_argument("--ckpt-dir", default=None)
    ap.add_argument("--out", default=None, help="write the tuned encoder (HF BERT names, safetensors)")
    args = ap.parse_args(argv)
    from ..engine.embed_engine import EmbeddingEngine
    from ..parallel.dist import init_distributed

    pctx = init_distributed()
    dev = str(pctx.device) if pctx.device.type == "cuda" else ("cuda" if torch.cuda.is_available() else "cpu")
    eng = EmbeddingEngine(args.model, device=dev)
    with open(args.data) as f:
        records = json.load(f)
    cfg = TrainConfig(lr=args.lr, max_steps=args.steps, micro_batch=args.micro_batch, global_batch=args.global_batch,
                      max_seq_len=512, warmup_steps=max(1, args.steps // 10))
    tr, params = embed_trainer(eng, records, cfg, args.hard_negatives, ckpt_dir=args.ckpt_dir)
    if args.ckpt_dir and tr.resume(args.ckpt_dir):
        print(f"resumed at step {tr.step}")
    tr.fit(args.steps - tr.step)
    if args.out and tr.rank == 0:
        from safetensors.torch import save_file

        Fn.write_back(eng.model, params, "encoder")
        os.makedirs(args.out, exist_ok=True)
        save_file({k: v.cpu().contiguous() for k, v in eng.model.state_dict().items()},
                  os.path.join(args.out, "model.safetensors"))


if __name__ == "__main__":
    main()
