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
* typed extraction (subject / subject type / relation / object / object type, the reference's
  5-tuples, utils/preprocessor.py:26-80) and the entities / relations / triples CSV export
  (utils/lc_graph.py:83-128);
* evaluation: :mod:`nv_genai_amd.experimental.kg_eval` (QA generation, the three answer modes,
  5-attribute reward scores, the reference's CSVs).
"""
from __future__ import annotations

import ast
import csv
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


# typed extraction: entity categories and relation verbs of the reference's extraction prompt
ENTITY_TYPES = ("ORG", "ORG/GOV", "ORG/REG", "PERSON", "GPE", "INSTITUTION", "PRODUCT", "EVENT", "FIELD",
                "METRIC", "TOOL", "CONCEPT")
RELATIONS = ("Has", "Announce", "Operate_In", "Introduce", "Produce", "Control", "Participates_In", "Impact",
             "Positive_Impact_On", "Negative_Impact_On", "Relate_To", "Is_Member_Of", "Invests_In", "Raise",
             "Decrease")
TYPED_EXTRACT_PROMPT = (
    "Extract knowledge-graph triples from the text as a Python list of tuples "
    "(head, head_type, relation, object, object_type). Entity types: " + ", ".join(ENTITY_TYPES) +
    ". Relations must be one of: " + ", ".join(RELATIONS) + ". Entities are specific names of at most "
    "three words (no dates, numbers or percentages); merge aliases of the same entity. Output only the list."
    "\n\nText:\n{text}")
TRIPLE_KEYS = ("subject", "subject_type", "relation", "object", "object_type")


def parse_typed_triples(text: str) -> List[Dict[str, str]]:
    """The LLM's list of 5-tuples (Python or JSON literal, possibly fenced) as dicts with the
    reference's keys; malformed tuples are skipped (process_response, preprocessor.py:26-43)."""
    m = re.search(r"\[.*\]", text, re.S)
    if not m:
        return []
    try:
        items = ast.literal_eval(m.group(0))
    except (ValueError, SyntaxError):
        try:
            items = json.loads(m.group(0))
        except json.JSONDecodeError:
            return []
    out = []
    for t in items if isinstance(items, (list, tuple)) else []:
        if isinstance(t, (list, tuple)) and len(t) == 5 and all(isinstance(x, str) and x.strip() for x in t):
            out.append(dict(zip(TRIPLE_KEYS, (x.strip() for x in t))))
    return out


def extract_typed_triples(text: str, llm) -> List[Dict[str, str]]:
    return parse_typed_triples(llm.invoke([("user", TYPED_EXTRACT_PROMPT.format(text=text))]))


def save_triples_to_csvs(triples: Sequence[Dict[str, str]], out_dir: str = ".") -> Dict[str, str]:
    """entities.csv (entity_id, entity_name, entity_type), relations.csv (relation_id,
    relation_name) and triples.csv (entity_id_1, relation_id, entity_id_2), ids in first-seen
    order; an entity's type is its type where it first appears as a subject, else as an
    object (lc_graph.py:83-128). Returns the three paths."""
    rel_ids: Dict[str, int] = {}
    for t in triples:
        rel_ids.setdefault(t["relation"], len(rel_ids))
    ent_ids: Dict[str, int] = {}
    for t in triples:
        ent_ids.setdefault(t["subject"], len(ent_ids))
    for t in triples:
        ent_ids.setdefault(t["object"], len(ent_ids))
    ent_type: Dict[str, str] = {}
    for t in triples:
        ent_type.setdefault(t["subject"], t["subject_type"])
    for t in triples:
        if t["object"] not in ent_type and t.get("object_type"):
            ent_type[t["object"]] = t["object_type"]
    os.makedirs(out_dir, exist_ok=True)
    paths = {k: os.path.join(out_dir, f"{k}.csv") for k in ("entities", "relations", "triples")}
    with open(paths["entities"], "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["entity_id", "entity_name", "entity_type"])
        for e, i in ent_ids.items():
            w.writerow([i, e, ent_type.get(e, "Unknown")])
    with open(paths["relations"], "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["relation_id", "relation_name"])
        for r, i in rel_ids.items():
            w.writerow([i, r])
    with open(paths["triples"], "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["entity_id_1", "relation_id", "entity_id_2"])
        for t in triples:
            w.writerow([ent_ids[t["subject"]], rel_ids[t["relation"]], ent_ids[t["object"]]])
    return paths


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

    def add_typed(self, triples: Iterable[Dict[str, str]]):
        for t in triples:
            s, o = t["subject"].lower(), t["object"].lower()
            self.g.add_edge(s, o, relation=t["relation"])
            self.g.nodes[s].setdefault("type", t.get("subject_type"))
            self.g.nodes[o].setdefault("type", t.get("object_type"))

    def entity_knowledge(self, entity: str, depth: int = 2) -> List[str]:
        """"subject relation object" along a depth-limited DFS from ``entity`` (LangChain's
        NetworkxEntityGraph.get_entity_knowledge, used by evaluation.py:98-135)."""
        import networkx as nx

        e = entity.lower()
        if not self.g.has_node(e):
            return []
        return [f"{a} {self.g[a][b]['relation']} {b}" for a, b in nx.dfs_edges(self.g, e, depth_limit=depth)]

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
