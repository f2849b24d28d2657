"""OpenAI/NIM-compatible model server on CPU with tiny models, exercised both through the
ASGI test client and through the real HTTP connectors (uvicorn on a loopback port)."""
import json
import socket
import threading
import time

import pytest
import torch


@pytest.fixture(scope="module")
def server():
    from nv_genai_amd.engine.embed_engine import EmbeddingEngine
    from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine
    from nv_genai_amd.serving.engine_service import EngineService
    from nv_genai_amd.serving.model_server import create_app

    eng = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=8, max_batched_tokens=512, max_model_len=512,
                                 kv_cache_blocks=64), device="cpu")
    svc = EngineService(eng)
    emb = EmbeddingEngine("encoder-tiny", device="cpu")
    rr = EmbeddingEngine("reranker-tiny", device="cpu")
    app = create_app(svc, emb, rr, llm_name="tiny-llm", embed_name="tiny-embed", rerank_name="tiny-rerank")
    yield app
    svc.shutdown()


@pytest.fixture(scope="module")
def client(server):
    from fastapi.testclient import TestClient

    with TestClient(server) as c:
        yield c


@pytest.fixture(scope="module")
def http_url(server):
    import uvicorn

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cfg = uvicorn.Config(server, host="127.0.0.1", port=port, log_level="error")
    srv = uvicorn.Server(cfg)
    t = threading.Thread(target=srv.run, daemon=True)
    t.start()
    for _ in range(200):
        if srv.started:
            break
        time.sleep(0.05)
    yield f"http://127.0.0.1:{port}"
    srv.should_exit = True
    t.join(timeout=5)


def test_models_and_health(client):
    ids = [m["id"] for m in client.get("/v1/models").json()["data"]]
    assert ids == ["tiny-llm", "tiny-embed", "tiny-rerank"]
    assert client.get("/v1/health/ready").status_code == 200
    assert client.get("/v1/health/live").status_code == 200


def test_chat_nonstream_deterministic(client):
    body = {"messages": [{"role": "user", "content": "hello there"}], "max_tokens": 6, "temperature": 0.0,
            "ignore_eos": True}
    a = client.post("/v1/chat/completions", json=body).json()
    b = client.post("/v1/chat/completions", json=body).json()
    assert a["object"] == "chat.completion"
    assert a["choices"][0]["message"]["content"] == b["choices"][0]["message"]["content"]
    assert a["usage"]["completion_tokens"] == 6
    assert a["choices"][0]["finish_reason"] == "length"


def test_chat_stream_frames(client):
    body = {"messages": [{"role": "user", "content": "stream please"}], "max_tokens": 5, "stream": True,
            "ignore_eos": True, "seed": 3}
    r = client.post("/v1/chat/completions", json=body)
    frames = [ln[6:] for ln in r.text.split("\n\n") if ln.startswith("data: ")]
    assert frames[-1] == "[DONE]"
    objs = [json.loads(f) for f in frames[:-1]]
    assert all(o["object"] == "chat.completion.chunk" for o in objs)
    # token frames carry one delta each, in the OpenAI chunk form, one id / created per stream
    assert len({(o["id"], o["created"]) for o in objs}) == 1
    assert all(o["choices"][0]["delta"]["role"] == "assistant" and o["choices"][0]["finish_reason"] is None
               for o in objs[:-1])
    assert objs[-1]["choices"][0]["finish_reason"] == "length"
    assert objs[-1]["usage"]["completion_tokens"] == 5


def test_completions(client):
    r = client.post("/v1/completions", json={"prompt": ["a b c", "d e"], "max_tokens": 3, "ignore_eos": True}).json()
    assert len(r["choices"]) == 2 and r["usage"]["completion_tokens"] == 6


def test_embeddings_query_passage_and_truncate(client):
    r = client.post("/v1/embeddings", json={"input": ["alpha beta", "gamma"], "input_type": "query"}).json()
    v = torch.tensor([d["embedding"] for d in r["data"]])
    assert v.shape == (2, 128)
    assert torch.allclose(v.norm(dim=1), torch.ones(2), atol=1e-4)
    p = client.post("/v1/embeddings", json={"input": "alpha beta", "input_type": "passage"}).json()
    assert not torch.allclose(torch.tensor(p["data"][0]["embedding"]), v[0])  # asymmetric prefix
    long = "word " * 2000
    assert client.post("/v1/embeddings", json={"input": long, "truncate": "NONE"}).status_code == 400
    assert client.post("/v1/embeddings", json={"input": long, "truncate": "END"}).status_code == 200
    b64 = client.post("/v1/embeddings", json={"input": "alpha", "encoding_format": "base64"}).json()
    assert isinstance(b64["data"][0]["embedding"], str)


def test_ranking(client):
    r = client.post("/v1/ranking", json={"query": {"text": "q"}, "passages": [{"text": "a"}, {"text": "b"}, {"text": "c"}]}).json()
    assert sorted(x["index"] for x in r["rankings"]) == [0, 1, 2]
    logits = [x["logit"] for x in r["rankings"]]
    assert logits == sorted(logits, reverse=True)


def test_http_connectors_roundtrip(http_url):
    from nv_genai_amd.connectors.http import ChatClient, EmbeddingsClient, RerankClient

    chat = ChatClient(http_url, "tiny-llm", max_tokens=4, temperature=0.0)
    streamed = "".join(chat.stream([("user", "hi")], ignore_eos=True))
    whole = chat.invoke([("user", "hi")], ignore_eos=True)
    assert streamed == whole
    # the async stream (what an async chain server forwards in the split topology) carries the
    # same text, per token or coalesced
    import asyncio

    from nv_genai_amd.connectors.http import _AIOHTTP_SESSIONS, aclose_clients

    async def agather(coalesce):
        out = [d async for d in chat.astream([("user", "hi")], coalesce=coalesce, ignore_eos=True)]
        sess = _AIOHTTP_SESSIONS[id(asyncio.get_running_loop())][1]
        await aclose_clients()          # what the chain server's lifespan runs at shutdown
        assert sess.closed
        return out

    per_tok = asyncio.run(agather(False))
    assert "".join(per_tok) == whole and len(per_tok) >= 2
    assert "".join(asyncio.run(agather(True))) == whole

    async def ahttpx():   # the httpx fallback (no aiohttp) carries the same text
        body = chat._body([("user", "hi")], True, ignore_eos=True)
        return [d async for d in chat._astream_httpx(f"{chat.base}/chat/completions", body, {}, False)]

    assert "".join(asyncio.run(ahttpx())) == whole
    emb = EmbeddingsClient(http_url, "tiny-embed")
    assert len(emb.embed_query("hello")) == 128
    assert len(emb.embed_documents(["a", "b", "c"])) == 3
    # batched query embeddings over base64: one request, the per-query vectors
    import torch

    qt = emb.embed_query_tensor(["hello", "world", "x"])
    assert qt.shape == (3, 128) and torch.allclose(qt[0], torch.tensor(emb.embed_query("hello")), atol=1e-6)
    rk = RerankClient(http_url, "tiny-rerank").rank("q", ["x", "y"])
    assert len(rk) == 2


def test_metrics_exposed(client):
    client.post("/v1/chat/completions", json={"model": "tiny-llm", "max_tokens": 2,
                                              "messages": [{"role": "user", "content": "hi"}]})
    t = client.get("/metrics").text
    assert "model_server_chat_requests_total" in t and "model_server_kv_usage" in t


def test_triton_generate_connector(http_url):
    from nv_genai_amd.connectors.triton import TritonLLM

    llm = TritonLLM(http_url.replace("http://", ""), model_name="ensemble", tokens=4, temperature=0.0)
    whole = llm.invoke("tell me", ignore_eos=True)
    streamed = "".join(llm.stream("tell me", ignore_eos=True))
    assert whole == streamed and isinstance(whole, str)


def test_router_proxies_and_balances(http_url):
    from fastapi.testclient import TestClient

    from nv_genai_amd.serving.router import create_router

    app = create_router([http_url, http_url + "/"])
    with TestClient(app) as c:
        assert [m["id"] for m in c.get("/v1/models").json()["data"]][0] == "tiny-llm"
        body = {"messages": [{"role": "user", "content": "hi"}], "max_tokens": 3, "ignore_eos": True,
                "temperature": 0.0}
        a = c.post("/v1/chat/completions", json=body).json()
        s = c.post("/v1/chat/completions", json=dict(body, stream=True)).text
        assert a["usage"]["completion_tokens"] == 3
        assert s.rstrip().endswith("data: [DONE]")
        st = c.get("/router/status").json()
        assert all(v == 0 for v in st["inflight"].values())


def test_beam_search_and_count_penalties(client):
    body = {"prompt": "beam me up", "max_tokens": 5, "ignore_eos": True, "beam_width": 3}
    a = client.post("/v1/completions", json=body).json()
    b = client.post("/v1/completions", json=body).json()
    assert a["choices"][0]["text"] == b["choices"][0]["text"]
    assert client.post("/v1/completions", json={**body, "beam_width": 99}).status_code == 422
    g = {"prompt": "x x x", "max_tokens": 12, "ignore_eos": True, "temperature": 0.0}
    plain = client.post("/v1/completions", json=g).json()["choices"][0]["text"]
    pen = client.post("/v1/completions", json={**g, "frequency_penalty": 2.0,
                                               "presence_penalty": 2.0}).json()["choices"][0]["text"]
    assert isinstance(pen, str) and client.post(
        "/v1/completions", json={**g, "presence_penalty": 3.0}).status_code == 422
    assert plain != pen or len(set(plain.split())) == len(plain.split())


def test_response_format_json_object(client):
    import json as _json

    body = {"messages": [{"role": "user", "content": "give me json"}], "max_tokens": 60,
            "response_format": {"type": "json_object"}, "seed": 1}
    r = client.post("/v1/chat/completions", json=body).json()
    txt = r["choices"][0]["message"]["content"]
    if r["choices"][0]["finish_reason"] == "stop":
        assert isinstance(_json.loads(txt), dict)
    else:
        assert txt.lstrip().startswith("{")


def test_n_choices_sampling_and_beams(client):
    body = {"messages": [{"role": "user", "content": "give me options"}], "max_tokens": 6, "ignore_eos": True,
            "n": 3, "temperature": 1.0, "seed": 7}
    r = client.post("/v1/chat/completions", json=body).json()
    assert [c["index"] for c in r["choices"]] == [0, 1, 2]
    texts = [c["message"]["content"] for c in r["choices"]]
    assert len(set(texts)) > 1 and r["usage"]["completion_tokens"] == 18
    again = client.post("/v1/chat/completions", json=body).json()
    assert [c["message"]["content"] for c in again["choices"]] == texts    # seeded per choice
    b = client.post("/v1/completions", json={"prompt": "beams", "max_tokens": 4, "ignore_eos": True,
                                             "beam_width": 3, "n": 2}).json()
    assert len(b["choices"]) == 2
    assert client.post("/v1/chat/completions", json={**body, "stream": True}).status_code == 400


def test_reference_connector_names_http_and_local(http_url):
    """The reference's client classes as drop-ins (connectors/compat.py): ChatNVIDIA /
    NVIDIAEmbeddings / NVIDIARerank and the LlamaIndex-style NVIDIA / NVIDIAEmbedding /
    LangchainEmbedding, over HTTP against the model server and in-process on the engines."""
    from types import SimpleNamespace

    from nv_genai_amd.connectors import compat
    from nv_genai_amd.engine.embed_engine import EmbeddingEngine
    from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine
    from nv_genai_amd.serving.engine_service import EngineService

    # HTTP (base_url as the reference passes it: http://host:port/v1)
    llm = compat.ChatNVIDIA(base_url=f"{http_url}/v1", model="tiny-llm", temperature=0.0, max_tokens=4)
    msg = llm.invoke("hello", ignore_eos=True)
    assert isinstance(msg, compat.AIMessage) and isinstance(msg.content, str)
    chunks = list(llm.stream([("system", "be brief"), ("user", "hello")], ignore_eos=True))
    whole = llm.invoke([("system", "be brief"), ("user", "hello")], ignore_eos=True)
    assert sum(chunks[1:], chunks[0]).content == whole.content
    assert len(llm.batch(["a", "b"], ignore_eos=True)) == 2
    emb_q = compat.NVIDIAEmbeddings(model="tiny-embed", base_url=f"{http_url}/v1")
    emb_p = compat.NVIDIAEmbeddings(model="tiny-embed", base_url=http_url, model_type="passage")
    q = emb_q.embed_query("alpha")
    assert len(q) == 128 and emb_p.embed_query("alpha") == emb_q.embed_documents(["alpha"])[0]
    docs = [SimpleNamespace(page_content=t, metadata={"source": i}) for i, t in enumerate(["x y", "z", "w v u"])]
    top = compat.NVIDIARerank(model="tiny-rerank", base_url=http_url, top_n=2).compress_documents(docs, "q")
    assert len(top) == 2 and all("relevance_score" in d.metadata and "source" in d.metadata for d in top)
    assert "relevance_score" not in docs[0].metadata          # inputs untouched
    li = compat.NVIDIA(model="tiny-llm", base_url=http_url, temperature=0.0, max_tokens=4)
    parts = list(li.stream_complete("hi", ignore_eos=True))
    assert parts[-1].text == li.complete("hi", ignore_eos=True).text == "".join(p.delta for p in parts)
    assert li.chat([compat.ChatMessage("user", "hi")], ignore_eos=True).message.role == "assistant"
    e = compat.LangchainEmbedding(emb_q, embed_batch_size=2)
    assert len(e.get_text_embedding_batch(["a", "b", "c"])) == 3
    assert e.get_query_embedding("alpha") == q

    # in-process: the same classes on the engines, no HTTP
    eng = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=4, max_batched_tokens=256, max_model_len=512,
                                 kv_cache_blocks=32), device="cpu")
    svc = EngineService(eng)
    try:
        local = compat.ChatNVIDIA(engine=svc, temperature=0.0, max_tokens=3)
        a = local.invoke("hello", ignore_eos=True).content
        assert "".join(c.content for c in local.stream("hello", ignore_eos=True)) == a
        assert local.bind(max_tokens=1).invoke("hello", ignore_eos=True).content == a[: len(
            local.bind(max_tokens=1).invoke("hello", ignore_eos=True).content)]
    finally:
        svc.shutdown()
    enc = EmbeddingEngine("encoder-tiny", device="cpu")
    le = compat.NVIDIAEmbedding(engine=enc)
    assert len(le.get_query_embedding("alpha")) == enc.dim
    rr = compat.NVIDIARerank(engine=EmbeddingEngine("reranker-tiny", device="cpu"), top_n=1)
    assert len(rr.compress_documents(docs, "q")) == 1


def test_sse_delta_parser_splits_lines_and_utf8_across_chunks():
    """The async chat stream's parser: frames cut anywhere (inside a line, inside a UTF-8
    character) come out whole; [DONE] ends the stream; non-data lines are skipped."""
    import json

    from nv_genai_amd.connectors.http import _sse_deltas

    frames = b"".join(b"data: " + json.dumps({"choices": [{"delta": {"content": t}}]}, ensure_ascii=False).encode()
                      + b"\n\n" for t in ["hé", "llo ", "世界"]) + b": keep-alive\n\ndata: [DONE]\n\n"
    for cut in range(1, len(frames)):
        carry, out, done = [b""], [], False
        for piece in (frames[:cut], frames[cut:]):
            parts, done = _sse_deltas(carry, piece)
            out += parts
            if done:
                break
        assert "".join(out) == "héllo 世界" and done, cut


def test_load_shedding_429_when_inflight_limit_reached(server, client):
    """max_inflight (NGA_MAX_INFLIGHT / --max-inflight): a generation request that would exceed
    the in-flight sequence limit gets 429 + Retry-After instead of an unbounded queue; n choices
    count as n sequences; under the limit requests run normally."""
    svc = server.state.llm
    body = {"messages": [{"role": "user", "content": "hi"}], "max_tokens": 2, "ignore_eos": True}
    old = server.state.max_inflight
    try:
        server.state.max_inflight = 2
        svc.handles[-99] = object()          # one sequence already in flight
        r = client.post("/v1/chat/completions", json={**body, "n": 2})
        assert r.status_code == 429 and r.headers["retry-after"] == "1"
        assert r.json()["error"]["type"] == "rate_limit_exceeded"
        assert client.post("/v1/completions", json={"prompt": ["a", "b"], "max_tokens": 2}).status_code == 429
        assert client.post("/v1/chat/completions", json=body).status_code == 200   # 1 + 1 <= 2
        assert "model_server_shed_requests_total" in client.get("/metrics").text
    finally:
        svc.handles.pop(-99, None)
        server.state.max_inflight = old
