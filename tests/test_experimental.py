"""Hybrid retrieval (RRF / outlier filter), knowledge-graph RAG (checkpoint/resume, graph
facts), on CPU with hash embeddings and a scripted LLM."""
import json

import pytest

from nv_genai_amd.connectors.fake import HashEmbeddings
from nv_genai_amd.index.vectorstore import VectorStore


def test_rrf_and_outliers():
    from nv_genai_amd.rag.hybrid import drop_outliers, rrf

    fused = rrf([[1, 2, 3], [3, 1, 4]], k=60)
    assert [d for d, _ in fused][:2] == [1, 3]
    assert abs(fused[0][1] - (1 / 61 + 1 / 62)) < 1e-12
    assert drop_outliers([10.0, 9.8, 2.0]) == [True, True, False]
    assert drop_outliers([1.0]) == [True]


def _store():
    st = VectorStore(HashEmbeddings(dim=128), dim=128, device="cpu")
    st.add_texts(["the mi355x gpu has 288 gb of hbm3e memory",
                  "llamas are domesticated south american camelids",
                  "rccl runs collectives over xgmi links between gpus",
                  "the weather today is sunny with light wind"],
                 [{"filename": f"f{i}.txt"} for i in range(4)])
    return st


def test_hybrid_retriever_sparse_dense_fusion():
    from nv_genai_amd.rag.hybrid import HybridRetriever

    st = _store()
    hr = HybridRetriever(st)
    top = hr.search("how much hbm3e memory does the mi355x have", k=2, pipeline="hybrid")
    assert top[0][0].page_content.startswith("the mi355x gpu")
    st.add_texts(["xgmi bandwidth is 153 gb/s per link"], [{"filename": "g.txt"}])
    top = hr.search("xgmi bandwidth per link", k=1, pipeline="hybrid")  # sync picks up the new doc
    assert "153" in top[0][0].page_content


def test_hybrid_ranked_uses_reranker():
    from nv_genai_amd.rag.hybrid import HybridRetriever

    class Rev:
        def rank(self, q, texts):
            return [{"index": i, "logit": float("weather" in t) * 10} for i, t in
                    sorted(enumerate(texts), key=lambda x: -float("weather" in x[1]))]

    hr = HybridRetriever(_store(), reranker=Rev())
    out = hr.search("gpu memory", k=3, pipeline="ranked_hybrid")
    assert len(out) == 1 and "weather" in out[0][0].page_content   # others dropped as outliers


class ScriptedLLM:
    def __init__(self, fail_on=None):
        self.calls = 0
        self.fail_on = fail_on

    def invoke(self, messages, **kw):
        self.calls += 1
        text = messages[-1][1]
        if self.fail_on and self.fail_on in text:
            raise RuntimeError("llm down")
        if "triples" in messages[0][1] or "triples" in text:
            if "mi355x" in text:
                return 'Sure: [["MI355X", "has", "HBM3E"], ["HBM3E", "capacity", "288 GB"]]'
            return '[["RCCL", "uses", "xGMI"]] trailing junk'
        return "answer: " + text[:40]


def test_kg_checkpoint_resume(tmp_path):
    from nv_genai_amd.experimental.knowledge_graph import build_graph, load_checkpoint

    docs = {"a.txt": ["the mi355x has hbm3e"], "b.txt": ["rccl over xgmi"]}
    ck = str(tmp_path / "ck.json")
    with pytest.raises(RuntimeError):
        build_graph(docs, ScriptedLLM(fail_on="rccl"), ck, workers=1)
    trip, done = load_checkpoint(ck)
    assert done == ["a.txt"] and len(trip) == 2                   # first document survived the crash
    llm = ScriptedLLM()
    kg = build_graph(docs, llm, ck, workers=2)
    assert llm.calls == 1                                           # resumed: only b.txt re-extracted
    assert set(kg.g.nodes) == {"mi355x", "hbm3e", "288 gb", "rccl", "xgmi"}
    # truncated checkpoint from a crashed non-atomic writer: complete triples are recovered
    (tmp_path / "bad.json").write_text('{"triples": [["a", "r", "b"], ["c", "r"')
    assert load_checkpoint(str(tmp_path / "bad.json")) == ([("a", "r", "b")], [])


def test_kg_rag_modes(tmp_path):
    from nv_genai_amd.experimental.knowledge_graph import KGRAG, KnowledgeGraph, parse_triples
    from nv_genai_amd.rag.hybrid import HybridRetriever

    kg = KnowledgeGraph()
    kg.add_triples(parse_triples('[["MI355X", "has", "HBM3E"], ["HBM3E", "capacity", "288 GB"]]'))
    assert kg.facts(["mi355x"]) == ["mi355x has hbm3e", "hbm3e capacity 288 gb"]   # 2 hops
    rag = KGRAG(kg, ScriptedLLM(), HybridRetriever(_store()))
    g = rag.context("what memory does the MI355X have?", mode="graph")
    assert "mi355x has hbm3e" in g and "Passages" not in g
    t = rag.context("what memory does the MI355X have?", mode="text")
    assert "Passages" in t and "facts" not in t
    c = rag.context("what memory does the MI355X have?", mode="combined")
    assert "facts" in c and "Passages" in c
    assert rag.answer("MI355X memory?").startswith("answer:")
