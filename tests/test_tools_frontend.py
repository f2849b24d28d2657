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
    assert c.post("/api/tts", json={"text": "x"}).status_code == 501   # speech is an optional remote service
    assert c.post("/api/asr", content=b"\0\0").status_code == 501


def test_frontend_speech_against_a_fake_speech_server(monkeypatch):
    """/api/asr and /api/tts through the real HTTP speech clients (dsp/asr.py, dsp/tts.py) to
    a local fake server with the OpenAI-style audio routes: a clip's segments come back as
    NDJSON transcripts, an answer comes back as streamed PCM16 (and as one WAV), segmented
    for the 300-character limit (reference tts_utils.py:105-108)."""
    import io
    import socket
    import threading
    import time
    import wave

    import numpy as np
    import uvicorn
    from fastapi import FastAPI, Request

    from nv_genai_amd.dsp.asr import pcm_to_wav
    from nv_genai_amd.frontend.api import create_frontend

    fake = FastAPI()
    seen = {"asr": [], "tts": []}

    @fake.post("/v1/audio/transcriptions")
    async def transcriptions(request: Request):
        from nv_genai_amd.chain_server.multipart import parse_multipart

        _, data = parse_multipart(await request.body(), request.headers.get("content-type", ""))["file"]
        with wave.open(io.BytesIO(data)) as w:
            n = w.getnframes()
        seen["asr"].append(n)
        return {"text": f"segment of {n} samples"}

    @fake.post("/v1/audio/speech")
    async def speech(request: Request):
        body = await request.json()
        seen["tts"].append(body["input"])
        pcm = (np.arange(len(body["input"]) * 100) % 200 - 100).astype("<i2").tobytes()
        return __import__("fastapi").Response(pcm_to_wav(pcm, 22050), media_type="audio/wav")

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    srv = uvicorn.Server(uvicorn.Config(fake, host="127.0.0.1", port=port, log_level="error"))
    t = threading.Thread(target=srv.run, daemon=True)
    t.start()
    try:
        for _ in range(200):
            if srv.started:
                break
            time.sleep(0.05)
        monkeypatch.setenv("SPEECH_API_URI", f"http://127.0.0.1:{port}")
        monkeypatch.setenv("SPEECH_ASR_SEGMENT_S", "1")
        c = TestClient(create_frontend(FakeChainClient()))
        assert c.get("/api/config").json()["speech"] is True
        clip = pcm_to_wav(np.zeros(16000 * 2 + 4000, dtype="<i2").tobytes(), 16000)   # 2.25 s
        lines = [json.loads(x) for x in c.post("/api/asr", content=clip).text.splitlines()]
        assert [x["text"] for x in lines] == ["segment of 16000 samples"] * 2 + ["segment of 4000 samples"]
        assert all(x["final"] for x in lines) and seen["asr"] == [16000, 16000, 4000]
        assert c.post("/api/asr?rate=8000", content=b"\0\0" * 10).status_code == 400   # wrong rate
        answer = "word " * 130                                                           # 650 characters
        r = c.post("/api/tts", json={"text": answer})
        assert r.status_code == 200 and r.headers["x-sample-rate"] == "22050"
        assert seen["tts"][-1].count(" . ") == 3                                        # segmented
        assert len(r.content) == 2 * 100 * len(seen["tts"][-1])
        w = c.post("/api/tts?format=wav", json={"text": "short answer"})
        with wave.open(io.BytesIO(w.content)) as wf:
            assert wf.getframerate() == 22050 and wf.getnframes() == 100 * len(seen["tts"][-1])
        assert c.post("/api/tts", json={"text": "  "}).status_code == 400
        # a RIFF header with a broken body is the client's error, not a server fault
        bad = b"RIFF" + (36).to_bytes(4, "little") + b"WAVEfmt " + b"\x10\x00\x00\x00" + b"\x07" * 16
        assert c.post("/api/asr", content=bad).status_code == 400
    finally:
        srv.should_exit = True
        t.join(timeout=5)


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
