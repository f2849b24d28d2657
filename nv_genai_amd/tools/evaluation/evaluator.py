"""RAG quality evaluation (tools/evaluation/rag_evaluator/evaluator.py, README.md:213-250).

The ``ragas`` package is not installed, so the six reported metrics are computed here with
this framework's own embedder and LLM (judge) — definitions follow RAGAS:

* answer_similarity  — cosine(embedding(answer), embedding(ground truth));
* answer_relevancy   — cosine(embedding(question), embedding(answer));
* faithfulness       — fraction of answer sentences the judge marks as supported by the
  retrieved context (falls back to token-overlap support when the judge output is unusable);
* context_precision  — rank-weighted precision of retrieved contexts relevant to the ground truth;
* context_relevancy  — fraction of context sentences that share content with the question;
* context_recall     — fraction of ground-truth sentences attributable to the retrieved context;
* ragas_score        — harmonic mean of faithfulness, context_relevancy, answer_relevancy,
  context_recall (as the reference computes it).
``eval_llm_judge`` is the Likert 1-5 judge with a JSON {"Rating", "Explanation"} reply.
Results go to ``<out>.json`` (means) and ``<out>.parquet`` / ``.csv`` (per sample).
"""
from __future__ import annotations

import json
import logging
import re
import statistics
from typing import Dict, List, Sequence

import torch

log = logging.getLogger(__name__)
_SENT = re.compile(r"(?<=[.!?])\s+")
_TOK = re.compile(r"[a-z0-9]+")
_STOP = {"the", "a", "an", "of", "and", "to", "in", "is", "are", "was", "for", "on", "with", "that", "this", "it", "as",
         "by", "be", "or", "at", "from", "what", "which", "who", "how"}

JUDGE_SYS = ("You are an impartial judge. Rate how well the answer responds to the question, using the reference "
             "context and reference answer. Reply ONLY with JSON: {\"Rating\": <integer 1-5>, \"Explanation\": \"...\"}")


def _sents(t: str) -> List[str]:
    return [s for s in _SENT.split(t.strip()) if s]


def _toks(t: str) -> set:
    return {w for w in _TOK.findall(t.lower()) if w not in _STOP}


def _overlap(a: str, b: str) -> float:
    ta = _toks(a)
    return len(ta & _toks(b)) / len(ta) if ta else 0.0


def _cos(emb, a: Sequence[str], b: Sequence[str]) -> List[float]:
    ea = torch.tensor(emb.embed_documents(list(a)), dtype=torch.float32)
    eb = torch.tensor(emb.embed_documents(list(b)), dtype=torch.float32)
    ea = ea / ea.norm(dim=1, keepdim=True).clamp_min(1e-9)
    eb = eb / eb.norm(dim=1, keepdim=True).clamp_min(1e-9)
    return (ea * eb).sum(1).tolist()


def _judge_supported(llm, statements: List[str], context: str) -> List[bool]:
    if llm is None or not statements:
        return [_overlap(s, context) >= 0.5 for s in statements]
    prompt = ("Context:\n" + context[:6000] + "\n\nFor each statement answer 1 if it can be inferred from the "
              "context, else 0. Reply ONLY with a JSON list of integers.\n" +
              "\n".join(f"{i + 1}. {s}" for i, s in enumerate(statements)))
    try:
        out = llm.invoke([("user", prompt)])
        m = re.search(r"\[[\s\d,]*\]", out)
        v = json.loads(m.group(0)) if m else []
        if len(v) == len(statements):
            return [bool(x) for x in v]
    except Exception as e:  # noqa: BLE001
        log.debug("judge failed: %s", e)
    return [_overlap(s, context) >= 0.5 for s in statements]


def ragas_metrics(samples: List[dict], emb, llm=None) -> List[Dict[str, float]]:
    qs = [s["question"] for s in samples]
    ans = [s.get("generated_answer", s.get("answer", "")) or " " for s in samples]
    gts = [s.get("ground_truth_answer", "") or " " for s in samples]
    sim = _cos(emb, ans, gts)
    rel = _cos(emb, qs, ans)
    rows = []
    for i, s in enumerate(samples):
        ctxs = s.get("retrieved_context") or []
        if isinstance(ctxs, str):
            ctxs = [ctxs]
        ctx = "\n".join(ctxs)
        a_sents = _sents(ans[i]) or [ans[i]]
        sup = _judge_supported(llm, a_sents, ctx)
        faith = sum(sup) / len(sup)
        rel_flags = [_overlap(gts[i], c) >= 0.3 for c in ctxs]
        hits, prec = 0, 0.0
        for k, f in enumerate(rel_flags, 1):
            if f:
                hits += 1
                prec += hits / k
        cprec = prec / hits if hits else 0.0
        c_sents = [x for c in ctxs for x in _sents(c)]
        crel = sum(_overlap(qs[i], x) > 0 for x in c_sents) / len(c_sents) if c_sents else 0.0
        g_sents = _sents(gts[i]) or [gts[i]]
        crec = sum(_overlap(g, ctx) >= 0.5 for g in g_sents) / len(g_sents)
        row = {"answer_similarity": sim[i], "faithfulness": faith, "context_precision": cprec,
               "context_relevancy": crel, "answer_relevancy": max(0.0, rel[i]), "context_recall": crec}
        parts = [row["faithfulness"], row["context_relevancy"], row["answer_relevancy"], row["context_recall"]]
        row["ragas_score"] = statistics.harmonic_mean(parts) if all(p > 0 for p in parts) else 0.0
        rows.append(row)
    return rows


def eval_ragas(eval_path: str, result_path: str, emb, llm=None) -> Dict[str, float]:
    with open(eval_path, encoding="utf-8") as fh:
        data = json.load(fh)
    rows = ragas_metrics(data, emb, llm)
    keys = list(rows[0]) if rows else []
    means = {k: statistics.fmean(r[k] for r in rows) for k in keys}
    parts = [means.get(k, 0.0) for k in ("faithfulness", "context_relevancy", "answer_relevancy", "context_recall")]
    means["ragas_score"] = statistics.harmonic_mean(parts) if parts and all(p > 0 for p in parts) else 0.0
    _write(result_path, data, rows, means)
    return means


def eval_llm_judge(eval_path: str, result_path: str, llm) -> Dict[str, float]:
    with open(eval_path, encoding="utf-8") as fh:
        data = json.load(fh)
    rows = []
    for d in data:
        prompt = (f"[Question]\n{d['question']}\n[The Start of Reference Context]\n{d.get('ground_truth_context', '')}\n"
                  f"[The End of Reference Context]\n[Reference Answer]\n{d.get('ground_truth_answer', '')}\n"
                  f"[Answer]\n{d.get('generated_answer', d.get('answer', ''))}")
        rating, expl = None, ""
        try:
            out = llm.invoke([("system", JUDGE_SYS), ("user", prompt)])
            m = re.search(r"\{.*\}", out, re.S)
            body = json.loads(m.group(0)) if m else {}
            rating = int(body.get("Rating"))
            expl = str(body.get("Explanation", body.get("Explanantion", "")))
        except Exception as e:  # noqa: BLE001
            expl = f"unparseable judge output: {e}"
        rows.append({"likert_rating": rating, "explanation": expl})
    valid = [r["likert_rating"] for r in rows if isinstance(r["likert_rating"], int)]
    means = {"mean_likert_rating": statistics.fmean(valid) if valid else 0.0, "rated": len(valid), "total": len(rows)}
    _write(result_path, data, rows, means)
    return means


def _write(result_path: str, data, rows, means):
    with open(result_path + ".json", "w", encoding="utf-8") as fh:
        json.dump(means, fh, indent=2)
    try:
        import pandas as pd

        df = pd.DataFrame([{**{k: v for k, v in d.items() if isinstance(v, (str, int, float))}, **r}
                           for d, r in zip(data, rows)])
        try:
            df.to_parquet(result_path + ".parquet")
        except Exception:  # noqa: BLE001 - no parquet engine: CSV instead
            df.to_csv(result_path + ".csv", index=False)
    except ImportError:
        pass
