"""Evaluation tool, RAG playground frontend (C13-C15) and the no-GPU
5-minute RAG (C16) on CPU with the deterministic fake backends."""
import json
import os

from fastapi.testclient import TestClient

from nv_genai_amd.connectors.fake import FakeChatModel, HashEmbeddings


class ScriptedLLM:
    """A judge / generator that answers from a fixed script (the fake backends of §4)."""

    def __init__(self, reply):
        self.reply = reply
        self.calls = []

    def invoke(self, messages, **kw):
        self.calls.append(messages)
        return self.reply(messages) if callable(self.reply) else self.reply

    def stream(self, messages, **kw):
        yield self.invoke(messages, **kw)


def test_ragas_metrics_rank_good_answers_above_bad(tmp_path):
    from nv_genai_amd.tools.evaluation.evaluator import eval_llm_judge, eval_ragas, ragas_metrics

    ctx = "Quartz City is the capital of the synthetic kingdom. The kingdom exports widgets."
    good = {"question": "What is the capital of the synthetic kingdom?",
            "generated_answer": "Quartz City is the capital of the synthetic kingdom.",
            "ground_truth_answer": "Quartz City is the capital of the synthetic kingdom.",
            "retrieved_context": [ctx], "ground_truth_context": ctx}
    bad = dict(good, generated_answer="Bananas grow on the moon every winter.",
               retrieved_context=["Unrelated text about rivers and mountains."])
    emb = HashEmbeddings(256)
    rows = ragas_metrics([good, bad], emb)
    for k in ("answer_similarity", "faithfulness", "context_precision", "context_recall", "ragas_score"):
        assert 0.0 <= rows[1][k] <= rows[0][k] <= 1.0 + 1e-6, k
    assert rows[0]["ragas_score"] > 0.0 and rows[1]["ragas_score"] == 0.0
    path = tmp_path / "eval.json"
    path.write_text(json.dumps([good, bad]))
    means = eval_ragas(str(path), str(tmp_path / "res"), emb)
    assert 0.0 < means["ragas_score"] <= 1.0
    judge = ScriptedLLM('Here is my verdict: {"Rating": 4, "Explanation": "mostly right"}')
    jm = eval_llm_judge(str(path), str(tmp_path / "judge"), judge)
    assert len(judge.calls) == 2 and jm["mean_likert_rating"] == 4 and jm["rated"] == 2


def test_synthetic_qa_generator_parses_pairs(tmp_path):
    from nv_genai_amd.tools.evaluation.data_generator import generate_synthetic_data

    docs = tmp_path / "docs"
    docs.mkdir()
    (docs / "a.txt").write_text("Widgets are made in Quartz City. " * 40)
    llm = ScriptedLLM('[{"question": "Where are widgets made?", "answer": "Quartz City"}, '
                      '{"question": "What is made in Quartz City?", "answer": "Widgets"}]')
    rows = generate_synthetic_data(str(docs), str(tmp_path / "qna.json"), llm)
    assert rows and {"question", "ground_truth_answer", "ground_truth_context", "document"} <= set(rows[0])
    assert json.loads((tmp_path / "qna.json").read_text()) == rows


class FakeChainClient:
    server_url = "http://chain:8081"
    model_name = "fake-llm"

    def __init__(self):
        self.docs = []

    def predict(self, query, use_knowledge_base, num_tokens=1024):
        yield from ["Quartz", " City", ""]

    def search(self, prompt, top_k=4):
        return [{"content": "Quartz City", "source": "facts.txt", "score": 0.9}][:top_k]

    def get_uploaded_documents(self):
        return list(self.docs)

    def delete_documents(self, name):
        self.docs.remove(name)
        return f"Deleted {name}"

    def upload_documents(self, paths):
        self.docs += [os.path.basename(p) for p in paths]


def test_frontend_pages_and_api():
    from nv_genai_amd.frontend.api import create_frontend

    fc = FakeChainClient()
    c = TestClient(create_frontend(fc))
    for page in ("/", "/content/converse", "/content/kb"):
        r = c.get(page)
        assert r.status_code == 200 and "Knowledge Base" in r.text
    assert c.get("/api/config").json()["model_name"] == "fake-llm"
    lines = [json.loads(x) for x in c.post("/api/generate", json={"query": "capital?"}).text.splitlines()]
    assert "".join(x["text"] for x in lines) == "Quartz City"
    assert c.post("/api/search", json={"query": "q", "top_k": 1}).json()[0]["source"] == "facts.txt"
    up = c.post("/api/documents", files={"file": ("facts.txt", b"Quartz City", "text/plain")})
    assert up.json()["message"] == "File uploaded successfully"
    assert c.get("/api/documents").json()["documents"] == ["facts.txt"]
    assert c.delete("/api/documents", params={"filename": "facts.txt"}).json()["message"] == "Deleted facts.txt"
    assert c.post("/api/tts").status_code == 501        # Riva is an optional remote service


def test_five_minute_rag_offline_and_reuse(tmp_path, capsys):
    from nv_genai_amd.examples.five_min_rag.main import main

    docs = tmp_path / "uploaded_docs"
    docs.mkdir()
    (docs / "kingdom.txt").write_text("Quartz City is the capital of the synthetic kingdom. " * 50)
    main(["--offline", "--docs", str(docs), "--store", str(tmp_path), "--question", "What is the capital?"])
    first = capsys.readouterr().out
    assert first.strip()
    assert os.path.exists(tmp_path / "vectorstore")
    main(["--offline", "--use-existing", "--docs", str(docs), "--store", str(tmp_path), "--question",
          "What is the capital?"])
    assert capsys.readouterr().out == first              # reused store answers identically


def test_fake_backends_are_deterministic():
    llm = FakeChatModel(words=5)
    assert llm.invoke([("user", "hi")]) == llm.invoke([("user", "hi")])
    emb = HashEmbeddings(64)
    assert emb.embed_query("a b") == emb.embed_query("a b")
