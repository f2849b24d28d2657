"""Knowledge-graph RAG (experimental/knowledge_graph_rag/).

* triple extraction: each text chunk is sent to the LLM, which returns JSON
  ``[["subject", "relation", "object"], ...]``; documents are processed with a worker pool
  and the extraction is **checkpointed after every document** (``{"triples",
  "processed_files"}`` JSON written atomically, resume skips processed files — the reference's
  construct_graph.py:46-111,178-210; a truncated checkpoint is recovered up to its last
  complete triple);
* graph: a ``networkx.DiGraph`` (cuGraph's role on the GPU is not needed at this scale);
* retrieval: entities of the question are matched against graph nodes, their 1-2 hop
  neighbourhood is rendered as "subject relation object" facts (graphRAG), the text store is
  searched with hybrid dense+BM25 RRF (textRAG), or both (combinedRAG);
* evaluation hook: answers of the three modes can be scored by any judge callable.
"""
from __future__ import annotations

import json
import logging
import os
import re
import tempfile
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Tuple

log = logging.getLogger(__name__)

EXTRACT_PROMPT = ("Extract knowledge-graph triples from the text. Reply ONLY with a JSON list of "
                  "[subject, relation, object] lists, using short noun phrases for entities.\n\nText:\n{text}")


def parse_triples(text: str) -> List[Tuple[str, str, str]]:
    out = []
    m = re.search(r"\[\s*\[.*\]\s*\]", text, re.S)
    if m:
        try:
            for t in json.loads(m.group(0)):
                if isinstance(t, list) and len(t) == 3 and all(isinstance(x, str) for x in t):
                    out.append((t[0].strip(), t[1].strip(), t[2].strip()))
            return out
        except json.JSONDecodeError:
            pass
    for a, b, c in re.findall(r'\[\s*"([^"]+)"\s*,\s*"([^"]+)"\s*,\s*"([^"]+)"\s*\]', text):
        out.append((a, b, c))
    return out


def save_checkpoint(triples: List[Sequence[str]], processed: List[str], path: str) -> None:
    d = os.path.dirname(os.path.abspath(path))
    fd, tmp = tempfile.mkstemp(dir=d, suffix=".tmp")
    with os.fdopen(fd, "w") as f:
        json.dump({"triples": [list(t) for t in triples], "processed_files": processed}, f)
    os.replace(tmp, path)


def load_checkpoint(path: str) -> Tuple[List[Tuple[str, str, str]], List[str]]:
    if not os.path.exists(path):
        return [], []
    with open(path) as f:
        content = f.read()
    try:
        d = json.loads(content)
        return [tuple(t) for t in d.get("triples", [])], list(d.get("processed_files", []))
    except json.JSONDecodeError:
        # truncated write from an older, non-atomic writer: keep every complete triple
        trip = [tuple(t) for t in json.loads("[" + ",".join(re.findall(r'\["[^"]*",\s*"[^"]*",\s*"[^"]*"\]', content)) + "]")]
        return trip, []


class KnowledgeGraph:
    def __init__(self):
        import networkx as nx

        self.g = nx.DiGraph()

    def add_triples(self, triples: Iterable[Sequence[str]]):
        for s, r, o in triples:
            self.g.add_edge(s.lower(), o.lower(), relation=r)

    def entities_in(self, text: str) -> List[str]:
        t = text.lower()
        return [n for n in self.g.nodes if len(n) > 2 and n in t]

    def facts(self, entities: Sequence[str], hops: int = 2, limit: int = 50) -> List[str]:
        seen, frontier, out = set(entities), list(entities), []
        for _ in range(hops):
            nxt = []
            for n in frontier:
                for _, o, d in self.g.out_edges(n, data=True):
                    out.append(f"{n} {d['relation']} {o}")
                    if o not in seen:
                        seen.add(o)
                        nxt.append(o)
                for s, _, d in self.g.in_edges(n, data=True):
                    out.append(f"{s} {d['relation']} {n}")
                    if s not in seen:
                        seen.add(s)
                        nxt.append(s)
            frontier = nxt
        return list(dict.fromkeys(out))[:limit]


def build_graph(docs: Dict[str, List[str]], llm, checkpoint: str, workers: int = 4,
                on_doc: Optional[Callable[[str], None]] = None) -> KnowledgeGraph:
    """docs: filename -> text chunks. Resumable: files already in the checkpoint are skipped."""
    triples, processed = load_checkpoint(checkpoint)
    todo = [f for f in docs if f not in processed]

    def extract(fname: str):
        out = []
        for chunk in docs[fname]:
            out += parse_triples(llm.invoke([("user", EXTRACT_PROMPT.format(text=chunk))]))
        return fname, out

    with ThreadPoolExecutor(max_workers=workers) as ex:
        for fname, trip in ex.map(extract, todo):
            triples += trip
            processed.append(fname)
            save_checkpoint(triples, processed, checkpoint)
            if on_doc:
                on_doc(fname)
    kg = KnowledgeGraph()
    kg.add_triples(triples)
    return kg


class KGRAG:
    """Answer with graph facts, text retrieval, or both (graphRAG / textRAG / combinedRAG)."""

    def __init__(self, kg: KnowledgeGraph, llm, hybrid=None):
        self.kg, self.llm, self.hybrid = kg, llm, hybrid

    def context(self, question: str, mode: str = "combined", k: int = 4) -> str:
        parts = []
        if mode in ("graph", "combined"):
            facts = self.kg.facts(self.kg.entities_in(question))
            if facts:
                parts.append("Knowledge graph facts:\n" + "\n".join(facts))
        if mode in ("text", "combined") and self.hybrid is not None:
            hits = self.hybrid.search(question, k, pipeline="hybrid")
            parts.append("Passages:\n" + "\n\n".join(d.page_content for d, _ in hits))
        return "\n\n".join(parts)

    def answer(self, question: str, mode: str = "combined") -> str:
        ctx = self.context(question, mode)
        return self.llm.invoke([("system", "Answer the question using only the provided context."),
                                ("user", f"{ctx}\n\nQuestion: {question}")])
