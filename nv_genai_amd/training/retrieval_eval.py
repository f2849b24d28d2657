"""Retriever evaluation: NDCG@k, MAP@k, Recall@k, Precision@k (the BEIR
``EvaluateRetrieval.evaluate`` step of retriever_customization.ipynb#cell 36, which reports
k = 1, 3, 5, 10, 100, 1000). Definitions follow pytrec_eval as BEIR uses it: graded
relevance, NDCG with log2 discount and linear gain, MAP@k normalised by min(#relevant, k).

``dense_retrieve`` runs the exact search with the in-HBM index kernels (score + radix top-k).
"""
from __future__ import annotations

import math
from typing import Dict, Sequence, Tuple

import torch

Qrels = Dict[str, Dict[str, int]]
Results = Dict[str, Dict[str, float]]


def evaluate(qrels: Qrels, results: Results, k_values: Sequence[int] = (1, 3, 5, 10, 100, 1000)
             ) -> Tuple[Dict[str, float], Dict[str, float], Dict[str, float], Dict[str, float]]:
    ndcg = {f"NDCG@{k}": 0.0 for k in k_values}
    _map = {f"MAP@{k}": 0.0 for k in k_values}
    recall = {f"Recall@{k}": 0.0 for k in k_values}
    prec = {f"P@{k}": 0.0 for k in k_values}
    qids = [q for q in qrels if q in results]
    for q in qids:
        rel = {d: r for d, r in qrels[q].items() if r > 0}
        ranked = [d for d, _ in sorted(results[q].items(), key=lambda x: (-x[1], x[0]))]
        ideal = sorted(rel.values(), reverse=True)
        for k in k_values:
            top = ranked[:k]
            dcg = sum(rel.get(d, 0) / math.log2(i + 2) for i, d in enumerate(top))
            idcg = sum(g / math.log2(i + 2) for i, g in enumerate(ideal[:k]))
            ndcg[f"NDCG@{k}"] += dcg / idcg if idcg > 0 else 0.0
            hits, ap = 0, 0.0
            for i, d in enumerate(top):
                if d in rel:
                    hits += 1
                    ap += hits / (i + 1)
            _map[f"MAP@{k}"] += ap / min(len(rel), k) if rel else 0.0
            recall[f"Recall@{k}"] += hits / len(rel) if rel else 0.0
            prec[f"P@{k}"] += hits / k
    n = max(1, len(qids))
    for m in (ndcg, _map, recall, prec):
        for key in m:
            m[key] = round(m[key] / n, 5)
    return ndcg, _map, recall, prec


def dense_retrieve(q_emb: torch.Tensor, p_emb: torch.Tensor, qids: Sequence[str], pids: Sequence[str],
                   k: int = 100) -> Results:
    from ..index.flat import FlatIndex

    index = FlatIndex(p_emb.shape[1], "ip", p_emb.device, capacity=p_emb.shape[0])
    index.add(p_emb)
    scores, ids = index.search(q_emb.to(p_emb.device), min(k, p_emb.shape[0]))
    scores, ids = scores.cpu().tolist(), ids.cpu().tolist()
    return {qids[i]: {pids[j]: s for j, s in zip(ids[i], scores[i]) if j >= 0} for i in range(len(qids))}
