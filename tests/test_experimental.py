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


# ---------------------------------------------------------------- KG-RAG evaluation (E4)
class EvalLLM:
    """QA generation, entity lists and answers for the evaluation pipeline."""

    def __init__(self):
        self.prompts = []

    def invoke(self, messages, **kw):
        text = messages[-1][1]
        self.prompts.append((messages[0][1][:40], text))
        if "synthetic evaluation data" in messages[0][1]:
            if "weather" in text:
                return "no json here"                    # dropped, like the reference
            return '```json\n{"question": "What memory does the MI355X have?", "answer": "288 GB of HBM3E."}\n```'
        if text.startswith("Return a JSON with a single key 'entities'"):
            return '{"entities": ["MI355X"]}' if "MI355X" in text else "not json"
        return "ANSWER(" + text.replace("\n", " ") + ")"


def test_typed_triples_csv_export(tmp_path):
    """entities / relations / triples CSVs of lc_graph.save_triples_to_csvs: ids in first-seen
    order, entity types from the first subject (else object) occurrence."""
    import csv

    from nv_genai_amd.experimental.knowledge_graph import KnowledgeGraph, parse_typed_triples, save_triples_to_csvs

    tr = parse_typed_triples("```[('AMD', 'ORG', 'Produce', 'MI355X', 'PRODUCT'), "
                             "('MI355X', 'PRODUCT', 'Has', 'HBM3E', 'PRODUCT'), ('bad', 'tuple'), "
                             "('AMD', 'ORG', 'Invests_In', 'ROCm', 'TOOL')]```")
    assert len(tr) == 3 and tr[0]["subject_type"] == "ORG"
    paths = save_triples_to_csvs(tr, str(tmp_path))
    ents = list(csv.DictReader(open(paths["entities"])))
    assert [(e["entity_id"], e["entity_name"], e["entity_type"]) for e in ents] == [
        ("0", "AMD", "ORG"), ("1", "MI355X", "PRODUCT"), ("2", "HBM3E", "PRODUCT"), ("3", "ROCm", "TOOL")]
    rels = list(csv.DictReader(open(paths["relations"])))
    assert [r["relation_name"] for r in rels] == ["Produce", "Has", "Invests_In"]
    trip = list(csv.DictReader(open(paths["triples"])))
    assert [(t["entity_id_1"], t["relation_id"], t["entity_id_2"]) for t in trip] == [("0", "0", "1"), ("1", "1", "2"),
                                                                                    ("0", "2", "3")]
    kg = KnowledgeGraph()
    kg.add_typed(tr)
    assert kg.entity_knowledge("amd") == ["amd Produce mi355x", "mi355x Has hbm3e", "amd Invests_In rocm"]
    assert kg.entity_knowledge("AMD", depth=1) == ["amd Produce mi355x", "amd Invests_In rocm"]
    assert kg.g.nodes["rocm"]["type"] == "TOOL"


def test_kg_evaluation_pipeline_writes_reference_csvs(tmp_path):
    """QA pairs -> text / graph / combined answers -> 5-attribute reward scores from the
    framework's reward model -> combined_results_with_scores.csv with the reference's columns
    (pages/evaluation.py:156-258)."""
    import csv

    from nv_genai_amd.experimental.kg_eval import KGEvaluator, create_qa_pairs, mean_scores, read_csv
    from nv_genai_amd.experimental.knowledge_graph import KnowledgeGraph
    from nv_genai_amd.models.reward import ATTRIBUTES, RewardModel
    from nv_genai_amd.rag.hybrid import HybridRetriever

    llm = EvalLLM()
    chunks = ["the mi355x gpu has 288 gb of hbm3e memory", "the weather today is sunny"]
    qa = create_qa_pairs(chunks, llm, num=2, out_csv=str(tmp_path / "qa_data.csv"))
    assert len(qa) == 1 and read_csv(str(tmp_path / "qa_data.csv")) == qa
    kg = KnowledgeGraph()
    kg.add_triples([("MI355X", "has", "HBM3E"), ("HBM3E", "capacity", "288 GB")])
    hr = HybridRetriever(_store())
    ev = KGEvaluator(kg, llm, search=lambda q, k: [d.page_content for d, _ in hr.search(q, k, pipeline="hybrid")])
    rows = ev.run(qa + [{"question": "How is the weather?", "answer": "sunny"}],
                  out_csv=str(tmp_path / "combined_results.csv"))
    with open(tmp_path / "combined_results.csv") as f:
        assert next(csv.reader(f)) == ["question", "gt_answer", "textRAG_answer", "graphRAG_answer", "combined_answer"]
    r0 = rows[0]
    assert "Here are the relevant passages from the knowledge base" in r0["textRAG_answer"]
    assert "relationships from the knowledge graph" in r0["graphRAG_answer"]
    ctx = [t for _, t in llm.prompts if t.startswith("Context: Here are the relevant") and "relationships" in t]
    assert ctx and "mi355x has hbm3e" in ctx[0] and "hbm3e capacity 288 gb" in ctx[0]     # depth-2 DFS
    assert "No graph triples were available" in rows[1]["graphRAG_answer"]            # entity JSON failed
    rm = RewardModel("reward-tiny", device="cpu", dtype=__import__("torch").float32)
    scored = ev.score(rows, rm, out_csv=str(tmp_path / "combined_results_with_scores.csv"))
    with open(tmp_path / "combined_results_with_scores.csv") as f:
        header = next(csv.reader(f))
    assert header[:5] == ["question", "gt_answer", "textRAG_answer", "graphRAG_answer", "combined_answer"]
    assert header[5:] == [f"{s}_{m}" for s in ("gt", "textRAG", "graphRAG", "combinedRAG") for m in ATTRIBUTES]
    vals = [float(scored[0][c]) for c in header[5:]]
    assert all(0.0 <= v <= 4.0 for v in vals) and len(set(vals)) > 1
    # one packed forward per row equals scoring each pair alone
    single = rm.score(rows[0]["question"], rows[0]["textRAG_answer"])
    assert all(abs(single[m] - scored[0][f"textRAG_{m}"]) < 1e-3 for m in ATTRIBUTES)
    ms = mean_scores(scored)
    assert set(ms) == {"gt", "textRAG", "graphRAG", "combinedRAG"} and set(ms["gt"]) == set(ATTRIBUTES)


def test_reward_endpoint_contract():
    """The model server answers the reward model's name with "helpfulness:x,..." content;
    RewardClient / parse_scores read it back (the reference's get_reward_scores format)."""
    import torch
    from fastapi.testclient import TestClient

    from nv_genai_amd.experimental.kg_eval import RewardClient
    from nv_genai_amd.models.reward import ATTRIBUTES, RewardModel, parse_scores
    from nv_genai_amd.serving.model_server import create_app

    rm = RewardModel("reward-tiny", device="cpu", dtype=torch.float32)
    app = create_app(None, None, None, reward=rm)
    with TestClient(app) as c:
        assert "nvidia/nemotron-4-340b-reward" in [m["id"] for m in c.get("/v1/models").json()["data"]]
        r = c.post("/v1/chat/completions", json={"model": "nvidia/nemotron-4-340b-reward", "messages": [
            {"role": "user", "content": "q?"}, {"role": "assistant", "content": "a."}]})
        assert r.status_code == 200
        sc = parse_scores(r.json()["choices"][0]["message"]["content"])
        want = rm.score("q?", "a.")
        assert sc is not None and all(abs(sc[m] - want[m]) < 1e-3 for m in ATTRIBUTES)
    assert parse_scores("garbage") is None
    assert RewardClient("http://127.0.0.1:9").base.startswith("http://127.0.0.1:9")
