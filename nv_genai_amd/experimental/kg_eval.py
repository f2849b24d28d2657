"""KG-RAG evaluation: text vs graph vs text+graph RAG, scored by a multi-attribute reward model
(experimental/knowledge_graph_rag/pages/evaluation.py, utils/preprocessor.py).

Pipeline, as the reference's evaluation page runs it:

1. :func:`create_qa_pairs` — sample document chunks, ask the LLM for one complex question /
   detailed answer pair per chunk as JSON (unparseable replies are dropped), write
   ``qa_data.csv`` (question, answer);
2. :meth:`KGEvaluator.run` — answer every question three ways, concurrently per question
   (three workers): **textRAG** (top-5 hybrid retrieval passages), **graphRAG** (the LLM lists
   the query's entities as JSON, each one's depth-2 graph neighbourhood becomes the context;
   when that fails a "no graph triples" disclaimer is the context), **combined** (both); all
   with the same "Envie" system prompt and "Context: ... \\n\\nUser query: ..." user turn; write
   ``combined_results.csv`` (question, gt_answer, textRAG_answer, graphRAG_answer,
   combined_answer);
3. :meth:`KGEvaluator.score` — the reward model scores the ground-truth answer and the three
   RAG answers of every question on helpfulness / correctness / coherence / complexity /
   verbosity; write ``combined_results_with_scores.csv`` with ``{gt,textRAG,graphRAG,
   combinedRAG}_{metric}`` columns.

The reward model is served by this framework (:class:`~nv_genai_amd.models.reward.RewardModel`
in process, or :class:`RewardClient` against the model server's chat route, the endpoint
contract of ``nvidia/nemotron-4-340b-reward``).
"""
from __future__ import annotations

import csv
import json
import os
import random
import re
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, Dict, List, Optional, Sequence

from ..models.reward import ATTRIBUTES, parse_scores
from .knowledge_graph import KnowledgeGraph

QA_SYSTEM = ("You generate synthetic evaluation data. From the passage you are given, write ONE hard question that "
             "needs most of the passage and several reasoning steps to answer, as a reader of the document would "
             "ask it, and a detailed, complete answer drawn only from the passage. Reply with JSON only: "
             '{"question": "...", "answer": "..."}.')
ENVIE_SYSTEM = ("You are a helpful AI assistant named Envie. You will reply to questions only based on the context "
                "that you are provided. If something is out of context, you will refrain from replying and politely "
                "decline to respond to the user.")
ENTITY_PROMPT = ("Return a JSON with a single key 'entities' and list of entities within this user query. Each element "
                 "in your list MUST BE part of the user's query. Do not provide any explanation. Here's the user "
                 "query: ")
NO_TRIPLES = ("No graph triples were available to extract from the knowledge graph. Always provide a disclaimer if "
              "you know the answer to the user's question, since it is not grounded in the knowledge you are provided "
              "from the graph.")
RESULT_COLUMNS = ("question", "gt_answer", "textRAG_answer", "graphRAG_answer", "combined_answer")
SCORE_COLUMNS = ("gt", "textRAG", "graphRAG", "combinedRAG")


def _json_obj(text: str):
    m = re.search(r"\{.*\}", text, re.S)
    return json.loads(m.group(0) if m else text)


def generate_qa_pair(text: str, llm) -> Optional[Dict[str, str]]:
    try:
        d = _json_obj(llm.invoke([("system", QA_SYSTEM), ("user", text)]))
    except (json.JSONDecodeError, TypeError):
        return None
    if not isinstance(d, dict) or "question" not in d or "answer" not in d:
        return None
    return {"question": str(d["question"]), "answer": str(d["answer"])}


def create_qa_pairs(chunks: Sequence[str], llm, num: int, seed: int = 0,
                    out_csv: Optional[str] = "qa_data.csv") -> List[Dict[str, str]]:
    rng = random.Random(seed)
    picks = rng.sample(list(chunks), min(num, len(chunks)))
    pairs = [p for p in (generate_qa_pair(c, llm) for c in picks) if p]
    if out_csv:
        _write(out_csv, ("question", "answer"), pairs)
    return pairs


def _write(path: str, cols: Sequence[str], rows: Sequence[Dict]) -> None:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(cols))
        w.writeheader()
        for r in rows:
            w.writerow({c: r.get(c, "") for c in cols})


def read_csv(path: str) -> List[Dict[str, str]]:
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


class RewardClient:
    """Reward scores from an OpenAI-compatible endpoint (this framework's model server with
    ``--reward``, or any server with the same contract): a chat completion over
    [user: question, assistant: answer] whose message content is "helpfulness:x,...".
    Returns None for an unusable reply, as the reference's get_reward_scores does."""

    def __init__(self, base_url: str, model: str = "nvidia/nemotron-4-340b-reward", timeout: float = 120.0):
        from ..connectors.http import _base

        self.base, self.model, self.timeout = _base(base_url), model, timeout

    def score(self, question: str, answer: str) -> Optional[Dict[str, float]]:
        import requests

        r = requests.post(f"{self.base}/chat/completions", timeout=self.timeout, json={
            "model": self.model, "messages": [{"role": "user", "content": question},
                                              {"role": "assistant", "content": answer}]})
        if r.status_code != 200:
            return None
        try:
            return parse_scores(r.json()["choices"][0]["message"]["content"])
        except (KeyError, IndexError, TypeError, ValueError):
            return None


class KGEvaluator:
    """``search(question, k) -> list of passage texts`` is the text retriever (the reference's
    hybrid BGE-M3 + reranker search, here e.g. :class:`~nv_genai_amd.rag.hybrid.HybridRetriever`)."""

    def __init__(self, kg: KnowledgeGraph, llm, search: Optional[Callable[[str, int], List[str]]] = None,
                 k: int = 5, depth: int = 2, workers: int = 3):
        self.kg, self.llm, self.search, self.k, self.depth, self.workers = kg, llm, search, k, depth, workers

    def _answer(self, context: str, question: str) -> str:
        return self.llm.invoke([("system", ENVIE_SYSTEM), ("user", "Context: " + context + "\n\nUser query: " + question)])

    def _passages(self, question: str) -> str:
        texts = self.search(question, self.k) if self.search is not None else []
        return "Here are the relevant passages from the knowledge base: \n\n" + "\n".join(texts)

    def _triples(self, question: str) -> str:
        ents = _json_obj(self.llm.invoke([("user", ENTITY_PROMPT + question)]))["entities"]
        trip: List[str] = []
        for e in ents:
            trip.extend(self.kg.entity_knowledge(str(e), depth=self.depth))
        return "Here are the relationships from the knowledge graph: " + "\n".join(trip)

    def text_answer(self, question: str) -> str:
        return self._answer(self._passages(question), question)

    def graph_answer(self, question: str) -> str:
        try:
            ctx = self._triples(question)
        except Exception:  # noqa: BLE001 - unparseable entity list: the reference's disclaimer
            ctx = NO_TRIPLES
        return self._answer(ctx, question)

    def combined_answer(self, question: str) -> str:
        try:
            ctx = self._passages(question) + "\n\n" + self._triples(question)
        except Exception:  # noqa: BLE001
            ctx = NO_TRIPLES
        return self._answer(ctx, question)

    def process_question(self, question: str, answer: str) -> Dict[str, str]:
        with ThreadPoolExecutor(max_workers=self.workers) as ex:
            ft = ex.submit(self.text_answer, question)
            fg = ex.submit(self.graph_answer, question)
            fc = ex.submit(self.combined_answer, question)
            return {"question": question, "gt_answer": answer, "textRAG_answer": ft.result(),
                    "graphRAG_answer": fg.result(), "combined_answer": fc.result()}

    def run(self, qa: Sequence[Dict[str, str]], out_csv: Optional[str] = "combined_results.csv",
            on_row: Optional[Callable[[int, Dict[str, str]], None]] = None) -> List[Dict[str, str]]:
        rows = []
        for i, p in enumerate(qa):
            rows.append(self.process_question(p["question"], p["answer"]))
            if on_row:
                on_row(i, rows[-1])
        if out_csv:
            _write(out_csv, RESULT_COLUMNS, rows)
        return rows

    @staticmethod
    def score(rows: Sequence[Dict[str, str]], reward, out_csv: Optional[str] = "combined_results_with_scores.csv"
              ) -> List[Dict]:
        """Reward scores of the ground truth and the three answers of every row. ``reward``
        has ``score(question, answer) -> dict | None`` (or ``score_batch``, used when present:
        one packed forward per row). A None score leaves that row's cells empty."""
        answer_cols = ("gt_answer", "textRAG_answer", "graphRAG_answer", "combined_answer")
        out = []
        for r in rows:
            q = r["question"]
            if hasattr(reward, "score_batch"):
                res = reward.score_batch([(q, r[c]) for c in answer_cols])
            else:
                res = [reward.score(q, r[c]) for c in answer_cols]
            row = dict(r)
            for st, sc in zip(SCORE_COLUMNS, res):
                for m in ATTRIBUTES:
                    row[f"{st}_{m}"] = "" if sc is None else sc[m]
            out.append(row)
        if out_csv:
            cols = list(RESULT_COLUMNS) + [f"{st}_{m}" for st in SCORE_COLUMNS for m in ATTRIBUTES]
            _write(out_csv, cols, out)
        return out


def mean_scores(rows: Sequence[Dict]) -> Dict[str, Dict[str, float]]:
    """Per answer set, the mean of each attribute (the reference's viz.png table)."""
    out = {}
    for st in SCORE_COLUMNS:
        out[st] = {}
        for m in ATTRIBUTES:
            v = [float(r[f"{st}_{m}"]) for r in rows if r.get(f"{st}_{m}") not in ("", None)]
            out[st][m] = round(sum(v) / len(v), 3) if v else float("nan")
    return out
