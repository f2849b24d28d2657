"""FM streaming-ASR RAG on CPU: filter design vs scipy, the DSP chain (reference ops),
stateful == whole-stream processing, FM round trip through UDP, ASR export, and the
alternate chain-server API (accumulator, time-window intents, summarisation)."""
import json
import socket
import threading
import time
from queue import Queue

import numpy as np
import pytest
import torch

from nv_genai_amd.connectors.fake import HashEmbeddings
from nv_genai_amd.index.vectorstore import VectorStore


def test_filter_design_matches_scipy():
    ss = pytest.importorskip("scipy.signal")
    from nv_genai_amd import ops
    from nv_genai_amd.dsp.design import decimator, firwin, reduce_fraction

    assert np.allclose(firwin(101, 100e3, 1e6), ss.firwin(101, 100e3, window="hamming", fs=1e6), atol=1e-12)
    assert reduce_fraction(1e6, 16e3) == (1, 62)
    d = decimator(62)
    x = np.random.default_rng(0).standard_normal(5887).astype(np.float32)
    ref = ss.resample_poly(x, 1, 62, window="hamming")
    y, _ = ops.resample_pcm(torch.from_numpy(x), torch.from_numpy(d.taps), d.down, d.pre, d.n_out(len(x)), 1.0)
    assert y.shape[0] == len(ref) and np.abs(y.numpy() - ref).max() < 1e-5


def test_fir_and_demod_reference_semantics():
    ss = pytest.importorskip("scipy.signal")
    from nv_genai_amd import ops

    rng = np.random.default_rng(1)
    x = (rng.standard_normal(3000) + 1j * rng.standard_normal(3000)).astype(np.complex64)
    taps = ss.firwin(101, 0.2, window="hamming")
    y = ops.fir_c64(torch.from_numpy(x), torch.tensor(taps, dtype=torch.float32)).numpy()
    assert np.abs(y - ss.lfilter(taps, [1.0], x)).max() < 1e-4
    d = ops.fm_demod(torch.from_numpy(x)).numpy()
    assert np.abs(d - np.diff(np.unwrap(np.angle(x)))).max() < 1e-4


def test_stateful_bursts_equal_whole_stream():
    from nv_genai_amd.dsp.replay import fm_modulate
    from nv_genai_amd.dsp.sdr import SDRPipeline

    t = np.arange(8000) / 16000
    audio = (0.4 * np.sin(2 * np.pi * 300 * t)).astype(np.float32)
    iq, _ = fm_modulate(audio, 16000, 1e6, deviation=30_000)
    whole = SDRPipeline(device="cpu", stateful=True).process(torch.from_numpy(iq))[0]
    p = SDRPipeline(device="cpu", stateful=True)
    parts = torch.cat([p.process(torch.from_numpy(iq[i:i + 5888]))[0] for i in range(0, len(iq), 5888)])
    n = min(len(whole), len(parts))
    assert n > 400 and torch.allclose(parts[:n], whole[:n], atol=1e-4)
    # the reference's stateless mode: one output block per burst, ceil(n_demod / 62) samples
    q = SDRPipeline(device="cpu")
    assert q.process(torch.from_numpy(iq[:5888]))[1].dtype == torch.int16
    assert q.process(torch.from_numpy(iq[:5888]))[0].numel() == -(-5887 // 62)


def test_udp_replay_receive_demodulates_tone(tmp_path):
    from nv_genai_amd.dsp.replay import replay, write_wav
    from nv_genai_amd.dsp.sdr import SDRPipeline, UDPReceiver

    fs = 16000
    t = np.arange(fs // 2) / fs
    write_wav(str(tmp_path / "tone.wav"), (0.5 * np.sin(2 * np.pi * 500 * t) * 32767).astype(np.int16), fs)
    q = Queue()
    rx = UDPReceiver(q, "127.0.0.1", 0, batch_size=47104)
    rx.start()
    n = replay(str(tmp_path / "tone.wav"), "127.0.0.1", rx.port, realtime=False)
    time.sleep(0.5)
    rx.stop()
    rx.join(timeout=2)
    bursts = []
    while not q.empty():
        bursts.append(q.get())
    assert n > 100 and len(bursts) >= 5
    p = SDRPipeline(device="cpu", stateful=True)
    y = torch.cat([p.process(torch.from_numpy(b))[0] for b in bursts]).numpy()[100:]
    f = np.fft.rfftfreq(len(y), 62 / 1e6)
    assert abs(f[np.abs(np.fft.rfft(y)).argmax()] - 500) < 10


def test_transcript_exporter_posts_finals_and_dedupes_partials():
    from nv_genai_amd.dsp.asr import ScriptedASR, TranscriptExporter

    class Sess:
        def __init__(self):
            self.posts = []

        def post(self, url, json=None, timeout=None):
            self.posts.append((url, json))

    s = Sess()
    q = Queue()
    for _ in range(20):
        q.put(b"\0\0" * 16000)           # 1 s of audio per chunk
    ex = TranscriptExporter(q, ScriptedASR("hello radio world. the weather is fine today. end", words_per_second=3),
                            database_uri="db:1", frontend_uri="fe:2", session=s)
    ex.start()
    time.sleep(1.0)
    ex.stop()
    ex.join(timeout=3)
    db = [j for u, j in s.posts if u.endswith("/storeStreamingText")]
    assert [d["transcript"] for d in db][:2] == ["hello radio world.", "the weather is fine today."]
    assert all(d["source_id"] == "Channel 0" for d in db)
    partials = [j["transcript"] for u, j in s.posts if u.endswith("update_running_transcript")]
    assert len(partials) == len(set(partials))


class IntentLLM:
    """Scripted LLM: intent/recency JSON (with the usual formatting mistakes), summaries, answers."""

    def __init__(self, intent, recency="{'timeNum': 5, 'timeUnit': 'min'}"):
        self.intent, self.recency, self.calls = intent, recency, []

    def invoke(self, messages, **kw):
        sys_, user = messages[0][1], messages[-1][1]
        self.calls.append(sys_[:40])
        if "classification system" in sys_:
            return f"Sure! Here is the JSON: {{'intentType': '{self.intent}'}}"
        if "restructuring natural language" in sys_:
            return self.recency
        if "summarization tool" in sys_:
            return "summary " + user[:20]
        return "answer"

    def stream(self, messages, **kw):
        yield self.invoke(messages)


@pytest.fixture
def fm_app():
    from nv_genai_amd.experimental import fm_asr

    def make(intent, **kw):
        store = VectorStore(HashEmbeddings(dim=64), 64, device="cpu")
        app = fm_asr.create_app(IntentLLM(intent, **kw), store, chunk_size=60, chunk_overlap=0)
        from fastapi.testclient import TestClient

        return app, TestClient(app)
    return make


def test_fm_chain_server_accumulates_and_answers(fm_app):
    app, c = fm_app("SpecificTopic")
    assert c.get("/serverStatus").json() == {"is_ready": True}
    r = c.post("/storeStreamingText", json={"transcript": "traffic on the bridge is heavy", "source_id": "ch0"})
    assert r.json() == {"status": "Added 0 entries"}
    for i in range(6):
        r = c.post("/storeStreamingText", json={"transcript": f"weather update number {i} says rain later today",
                                                "source_id": "ch0"})
    assert int(r.json()["status"].split()[1]) >= 1
    body = json.dumps({"question": "what about the weather?", "max_docs": 3})
    out = c.request("GET", "/generate", content=body).text
    assert out.startswith("*Returned") and out.endswith("answer")


def test_fm_recent_summary_and_time_window(fm_app):
    from nv_genai_amd.experimental import fm_asr

    app, c = fm_app("RecentSummary")
    acc = app.state.accumulator
    old = fm_asr.dt.datetime.now() - fm_asr.dt.timedelta(minutes=30)
    acc.db.insert_docs(["an old entry"], "ch0", tnow=old)
    acc.db.insert_docs([f"recent entry {i}" for i in range(8)], "ch0")
    body = json.dumps({"question": "summarize the last 5 minutes", "max_docs": 3, "allow_summary": True})
    out = c.request("GET", "/generate", content=body).text
    assert out.startswith("*Found 8 entries from the last 300s*") and "summarization" in out
    app2, c2 = fm_app("TimeWindow", recency='{"timeNum": 30, "timeUnit": "minutes"}')
    app2.state.accumulator.db.insert_docs(["an old entry"], "ch0", tnow=old)
    out = c2.request("GET", "/generate", content=json.dumps({"question": "what was said 30 minutes ago?"})).text
    assert out.startswith("*Found 1 entries from 1800s ago")


def test_fm_plain_chat_and_unknown_intent(fm_app):
    app, c = fm_app("Unknown")
    out = c.request("GET", "/generate", content=json.dumps({"question": "hi", "use_knowledge_base": False})).text
    assert out == "answer"
    out = c.request("GET", "/generate", content=json.dumps({"question": "anything?"})).text
    assert out == "*Found no documents related to the query*"
