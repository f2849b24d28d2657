"""Hard-negative mining for retriever fine-tuning (SURVEY.md §2.B K17, §2.A E8;
experimental/synthetic-data-retriever-customization/retriever_customization.ipynb#cell 21-24).

For each query: score every passage (q·pᵀ), take the *minimum* score over the query's
positives, and keep as candidates only passages that are not positives and score at most
``margin × min_pos`` (passages scoring close to or above a positive are likely unlabelled
positives); the ``num_negs`` best-scoring candidates are the hard negatives.

On the GPU the scores come from the skinny MFMA score kernel and the selection from the
radix top-k kernel of the vector index (``ops.score`` / ``ops.topk``), one query block at a
time so the [Q, N] score matrix never exceeds ``block`` rows. The reference returns
``np.argpartition`` order (unsorted); here negatives are sorted by score, best first.
"""
from __future__ import annotations

from typing import List, Sequence

import torch

from .. import ops


def mine_hard_negatives(q: torch.Tensor, p: torch.Tensor, positives: Sequence[Sequence[int]],
                        margin: float = 0.95, num_negs: int = 10, block: int = 1024) -> List[List[int]]:
    """q [Q, D], p [N, D] (any float dtype, same device); positives[i] = passage ids of query i."""
    Q, N = q.shape[0], p.shape[0]
    out: List[List[int]] = []
    gpu = q.is_cuda
    pb = p.to(torch.bfloat16).contiguous() if gpu else p.float()
    for s in range(0, Q, block):
        qb = q[s:s + block]
        if gpu:
            scores = ops.score(qb.to(torch.bfloat16).contiguous(), pb)          # [b, N] fp32
        else:
            scores = qb.float() @ pb.t()
        b = scores.shape[0]
        rows = torch.arange(b, device=scores.device)
        pos_r = torch.tensor([r for r in range(b) for _ in positives[s + r]], dtype=torch.long,
                             device=scores.device)
        pos_c = torch.tensor([c for r in range(b) for c in positives[s + r]], dtype=torch.long,
                             device=scores.device)
        pos_s = scores[pos_r, pos_c]
        min_pos = torch.full((b,), float("inf"), device=scores.device).scatter_reduce(
            0, pos_r, pos_s, reduce="amin")
        thr = min_pos * margin
        scores[pos_r, pos_c] = float("-inf")
        scores = scores.masked_fill(scores > thr[:, None], float("-inf"))
        k = min(num_negs, N)
        if gpu:
            vals, idx = ops.topk(scores, k)
        else:
            vals, idx = scores.topk(k, dim=1)
        vals, idx = vals.cpu(), idx.cpu()
        for r in range(b):
            out.append([int(i) for v, i in zip(vals[r].tolist(), idx[r].tolist()) if v != float("-inf")])
        del rows
    return out


def build_training_records(queries: Sequence[str], passages: Sequence[str], positives: Sequence[Sequence[int]],
                           negatives: Sequence[Sequence[int]]) -> List[dict]:
    """The NeMo SBERT fine-tuning JSON records: {"question", "pos_doc": [...], "neg_doc": [...]}."""
    return [{"question": q, "pos_doc": [passages[i] for i in pos], "neg_doc": [passages[i] for i in neg]}
            for q, pos, neg in zip(queries, positives, negatives)]
