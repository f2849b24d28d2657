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


class ListLLM:
    """Answers multi-query prompts with a list, everything else with a fixed string."""

    def __init__(self):
        self.prompts = []

    def stream(self, messages, **kw):
        yield self.invoke(messages)

    def invoke(self, messages, **kw):
        text = messages[-1][1]
        self.prompts.append(text)
        if "different versions" in text:
            return "Here are the questions:\n1. hbm3e capacity of mi355x\n2) xgmi links between gpus\n\n- llamas"
        if "summarize" in text:
            return "summary: user asked about gpus"
        if "[[RESPONSE]]" in text:
            return "**:green[TRUE]** supported"
        if "rewrite" in messages[0][1] if len(messages) > 1 else False:
            return "rewritten: how much memory does the mi355x have"
        return "the gpu memory is large"


def test_parse_lines_and_dedupe():
    from nv_genai_amd.rag.advanced import dedupe, parse_lines, sources_of
    from nv_genai_amd.index.vectorstore import Document

    assert parse_lines("Here are:\n1. a\n2) b\n\n- c\n") == ["a", "b", "c"]
    docs = [Document("x", {"source": "s1"}), Document("x", {"source": "s2"}), Document("y", {"source": "s1"})]
    d = dedupe(docs)
    assert [x.metadata["source"] for x in d] == ["s1", "s1"]
    assert sources_of(d)["s1"]["doc_content"] == "x\n\ny"


def test_advanced_retriever_modes():
    from nv_genai_amd.rag.advanced import AdvancedRetriever

    class Rev:
        def rank(self, q, texts):
            return [{"index": i, "logit": -i} for i in range(len(texts))][::-1]

    st = _store()
    llm = ListLLM()
    r = AdvancedRetriever(st, llm, Rev(), k=4, score_threshold=0.0, top_n=2)
    d0, ctx0, _ = r.retrieve("hbm3e memory of the mi355x", 0)
    assert len(d0) == 4 and ctx0.count("\n\n") == 4
    d1, _, src1 = r.retrieve("hbm3e memory", 1)
    assert len(d1) == 2 and len({x.page_content for x in d1}) == 2          # deduped + reranked top-2
    d2, _, _ = r.retrieve("hbm3e memory", 2)
    assert any("the gpu memory is large" in p for p in llm.prompts) or len(d2) == 2
    with pytest.raises(ValueError):
        r.retrieve("q", 9)


def test_merger_and_embedding_filters():
    from nv_genai_amd.index.vectorstore import Document
    from nv_genai_amd.rag.advanced import (ContextualCompressionRetriever, EmbeddingsFilter,
                                           EmbeddingsRedundantFilter, MergerRetriever)

    class R:
        def __init__(self, docs):
            self.docs = docs

        def invoke(self, q):
            return self.docs

    a = [Document("gpu memory hbm3e"), Document("llamas")]
    b = [Document("gpu memory hbm3e"), Document("xgmi links"), Document("weather")]
    merged = MergerRetriever([R(a), R(b)]).invoke("q")
    assert [d.page_content for d in merged] == ["gpu memory hbm3e", "gpu memory hbm3e", "llamas", "xgmi links",
                                                "weather"]
    emb = HashEmbeddings(dim=128)
    uniq = EmbeddingsRedundantFilter(emb).transform_documents(merged)
    assert len(uniq) == 4
    comp = ContextualCompressionRetriever(MergerRetriever([R(a), R(b)]),
                                          [EmbeddingsRedundantFilter(emb), EmbeddingsFilter(emb, 0.99)])
    assert [d.page_content for d in comp.invoke("gpu memory hbm3e")] == ["gpu memory hbm3e"]


def test_advanced_chat_turn_memory_factcheck_feedback(tmp_path):
    from nv_genai_amd.rag.advanced import AdvancedRAGChat, AdvancedRetriever, FeedbackLog

    llm = ListLLM()
    chat = AdvancedRAGChat(AdvancedRetriever(_store(), llm, None, k=2, score_threshold=0.0), llm, "You are ORAN bot")
    out = chat.ask("what memory does the mi355x have")
    assert out["answer"] == "the gpu memory is large" and out["fact_check"].startswith("**:green[TRUE]**")
    assert chat.memory.buffer.startswith("summary")
    out2 = chat.ask("and how fast is it?")                 # follow-up is rewritten against the summary
    assert out2["query"].startswith("rewritten")
    fb = FeedbackLog(str(tmp_path / "fb.jsonl"))
    row = fb.submit({"score": "🙂", "text": "ok"}, "q", "r")
    assert row["score"] == 4 and json.loads((tmp_path / "fb.jsonl").read_text())["comment"] == "Score: 4/5. Feedback: ok"
