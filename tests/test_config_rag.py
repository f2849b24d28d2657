"""Config wizard (APP_* parity), loaders / splitters, vector store / IVF / persistence,
tracing propagation."""
import io
import json
import os
import zipfile

import pytest
import torch

from nv_genai_amd.chain_server.configuration import AppConfig


def test_env_names_match_reference_scheme():
    names = {n for n, _, _ in AppConfig.envvars()}
    for n in ("APP_VECTORSTORE_URL", "APP_VECTORSTORE_NLIST", "APP_LLM_MODELNAME", "APP_LLM_SERVERURL",
              "APP_TEXTSPLITTER_CHUNKSIZE", "APP_TEXTSPLITTER_CHUNKOVERLAP", "APP_EMBEDDINGS_DIMENSIONS",
              "APP_RETRIEVER_SCORETHRESHOLD", "APP_RETRIEVER_TOPK", "APP_PROMPTS_RAGTEMPLATE",
              "APP_PROMPTS_CHATTEMPLATE", "APP_EMBEDDINGS_SERVERURL", "APP_ENGINE_TPSIZE", "APP_INDEX_TYPE"):
        assert n in names


def test_defaults():
    c = AppConfig.from_dict({})
    assert c.vector_store.nlist == 64 and c.vector_store.nprobe == 16
    assert c.text_splitter.chunk_size == 510 and c.text_splitter.chunk_overlap == 200
    assert c.retriever.top_k == 4 and c.retriever.score_threshold == 0.25
    assert c.embeddings.dimensions == 1024
    assert "{context_str}" in c.prompts.rag_template


def test_env_json_decoding_and_file_precedence(tmp_path, monkeypatch):
    monkeypatch.setenv("APP_RETRIEVER_TOPK", "7")
    monkeypatch.setenv("APP_LLM_MODELNAME", "meta/llama3-70b-instruct")
    monkeypatch.setenv("APP_VECTORSTORE_URL", "http://other:1")
    f = tmp_path / "cfg.yaml"
    f.write_text("vectorStore:\n  url: http://file:19530\nretriever:\n  scoreThreshold: 0.5\n")
    c = AppConfig.from_file(str(f))
    assert c.retriever.top_k == 7                       # env fills an unset key (JSON-decoded to int)
    assert c.llm.model_name == "meta/llama3-70b-instruct"
    assert c.vector_store.url == "http://file:19530"    # file wins over env (reference quirk)
    assert c.retriever.score_threshold == 0.5
    jf = tmp_path / "cfg.json"
    jf.write_text(json.dumps({"llm": {"model_engine": "local"}}))
    assert AppConfig.from_file(str(jf)).llm.model_engine == "local"
    bad = tmp_path / "bad.yaml"
    bad.write_text("{:::")
    assert AppConfig.from_file(str(bad)) is None
    assert AppConfig.from_file(str(tmp_path / "missing.yaml")) is None


def test_print_help():
    out = []
    AppConfig.print_help(out.append)
    text = "".join(out)
    assert "ENV Variable: APP_VECTORSTORE_URL" in text and "chunkSize: 510" in text


def test_loaders_pdf_pptx_html(tmp_path):
    from nv_genai_amd.rag.loaders import load_file, make_pdf

    p = tmp_path / "doc.pdf"
    p.write_bytes(make_pdf(["Alpha page text", "Beta page (with parens)"]))
    docs = load_file(str(p))
    assert [d.page_content for d in docs] == ["Alpha page text", "Beta page (with parens)"]
    assert docs[1].metadata["page"] == 2
    pp = tmp_path / "deck.pptx"
    with zipfile.ZipFile(pp, "w") as z:
        for i, t in enumerate(["Slide one", "Slide two"], 1):
            z.writestr(f"ppt/slides/slide{i}.xml",
                       f'<p:sld xmlns:p="p" xmlns:a="a"><a:t>{t}</a:t></p:sld>')
    assert [d.page_content for d in load_file(str(pp))] == ["Slide one", "Slide two"]
    h = tmp_path / "x.html"
    h.write_text("<html><script>bad()</script><p>Hello</p><p>World</p></html>")
    assert load_file(str(h))[0].page_content.split() == ["Hello", "World"]
    with pytest.raises(ValueError):
        load_file(str(tmp_path / "file.xyz"))


def test_token_splitter_overlap():
    from nv_genai_amd.rag.splitters import TokenTextSplitter

    s = TokenTextSplitter(tokens_per_chunk=20, chunk_overlap=5)
    text = " ".join(f"word{i}" for i in range(200))
    chunks = s.split_text(text)
    assert len(chunks) > 5 and all(s.count_tokens(c) <= 22 for c in chunks)
    assert chunks[0].split()[-1] in chunks[1]  # overlap carries context forward


def test_vectorstore_flat_ivf_and_persistence(tmp_path):
    from nv_genai_amd.connectors.fake import HashEmbeddings
    from nv_genai_amd.index.vectorstore import VectorStore

    emb = HashEmbeddings(128)
    texts = [f"document about topic {i} with keyword k{i % 7}" for i in range(300)]
    metas = [{"filename": f"f{i % 3}.txt"} for i in range(300)]
    for itype in ("flat", "ivf_flat", "hnsw"):
        vs = VectorStore(emb, 128, itype, "cosine", "cpu", nlist=8, nprobe=8, persist_dir=str(tmp_path / itype))
        vs.add_texts(texts, metas)
        hits = vs.similarity_search_with_score("topic 42 keyword k0", 3)
        assert "topic 42 " in hits[0][0].page_content
        assert sorted(vs.get_filenames()) == ["f0.txt", "f1.txt", "f2.txt"]
        assert vs.delete_by_filename("f0.txt")
        assert all(d.metadata["filename"] != "f0.txt" for d, _ in vs.similarity_search_with_score("topic 42 k0", 20))
        vs2 = VectorStore(emb, 128, itype, "cosine", "cpu", persist_dir=str(tmp_path / itype))
        assert len(vs2) == 200
        assert vs2.similarity_search("topic 43 keyword k1", 1)[0].page_content == texts[43]
        rel = vs2.similarity_search_with_relevance_scores("topic 43 keyword k1", 4, score_threshold=0.25)
        assert rel and all(s >= 0.25 for _, s in rel)


def test_synthetic_collection_whitens_a_remote_encoder(monkeypatch):
    """The REST benchmark corpus over an encoder behind HTTP (split topology): the chain server
    whitens the remote query vectors (nearly collinear from a random-init encoder) so concurrent
    questions retrieve different chunks, as the in-process engine's own whitening does."""
    from nv_genai_amd.chain_server import utils
    from nv_genai_amd.engine.embed_engine import pca_whitening
    from nv_genai_amd.index.vectorstore import VectorStore, WhitenedEmbedder

    class Remote:   # the EmbeddingsClient surface the store uses: collinear-ish query vectors
        dim = 64

        def __init__(self):
            self.base = torch.randn(64)

        def embed_query_tensor(self, texts):
            g = torch.Generator().manual_seed(abs(hash(tuple(texts))) % (2 ** 31))
            return self.base + 0.01 * torch.randn(len(texts), 64, generator=g)

    cfg = AppConfig.from_dict({"index": {"synthetic_docs": 2000}, "embeddings": {"model_engine": "nim"}})
    vs = VectorStore(Remote(), 64, "flat", "cosine", "cpu", batch_queries=False)
    utils._fill_synthetic(vs, cfg)
    assert isinstance(vs.embedder, WhitenedEmbedder)
    qs = [f"question {i} about widgets" for i in range(64)]
    y = torch.cat([vs.embedder.embed_query_tensor([q]) for q in qs])
    assert torch.allclose(y.norm(dim=1), torch.ones(64), atol=1e-4)
    raw = torch.cat([vs.embedder.inner.embed_query_tensor([q]) for q in qs])
    raw = raw / raw.norm(dim=1, keepdim=True)
    off = ~torch.eye(64, dtype=torch.bool)
    assert (raw @ raw.T)[off].mean() > 0.99            # unwhitened: every question alike
    assert (y @ y.T)[off].abs().mean() < 0.3           # whitened: spread out
    firsts = {vs.similarity_search_with_score(q, 4)[0][0].page_content for q in qs}
    assert len(firsts) > 32                             # different questions, different chunks
    mu, W = pca_whitening(torch.randn(500, 8))
    assert mu.shape == (8,) and W.shape == (8, 8)


def test_flat_l2_and_ip_metrics():
    from nv_genai_amd.index.flat import FlatIndex

    g = torch.Generator().manual_seed(1)
    X = torch.randn(500, 32, generator=g)
    q = torch.randn(3, 32, generator=g)
    for metric in ("l2", "ip"):
        idx = FlatIndex(32, metric, "cpu")
        idx.add(X, torch.arange(500) + 1000)
        v, i = idx.search(q, 5)
        qb = q.bfloat16().float()  # queries are scored in bf16, like the stored vectors
        if metric == "l2":
            d = (qb * qb).sum(1, keepdim=True) - 2 * qb @ X.bfloat16().float().T \
                + X.bfloat16().float().pow(2).sum(1)[None]
            rv, ri = torch.topk(-d, 5)
        else:
            rv, ri = torch.topk(qb @ X.bfloat16().float().T, 5)
        assert torch.equal(i, ri + 1000)
        assert torch.allclose(v, rv, atol=0.1)  # |q|^2 is added back from the fp32 query


def test_tracing_traceparent_propagation():
    from nv_genai_amd.observability.tracing import InMemoryExporter, Tracer, inject_context

    exp = InMemoryExporter()
    fe = Tracer("frontend", exp, enabled=True)
    cs = Tracer("chain-server", exp, enabled=True)
    with fe.span("predict") as s:
        hdr = inject_context()
    with cs.span("POST /generate", traceparent=hdr["traceparent"]) as c:
        with cs.span("retriever"):
            pass
    names = {sp.name: sp for sp in exp.spans}
    assert names["POST /generate"].trace_id == names["predict"].trace_id
    assert names["POST /generate"].parent_id == names["predict"].span_id
    assert names["retriever"].parent_id == names["POST /generate"].span_id


def test_reference_style_vector_clients():
    """MilvusVectorClient / QdrantVectorClient contract (experimental/multimodal_assistant/
    retriever/vector.py) over the in-HBM indices."""
    import torch

    from nv_genai_amd.index.clients import MilvusStyleClient, QdrantStyleClient, drop_collection
    from nv_genai_amd.index.vectorstore import Document

    g = torch.Generator().manual_seed(0)
    docs = [Document(f"content {i}", {"source": f"file{i}.pdf", "page_num": i}) for i in range(300)]
    emb = torch.randn(300, 32, generator=g)
    for cls, first in ((MilvusStyleClient, 0), (QdrantStyleClient, 1)):
        name = f"test_{cls.__name__}"
        drop_collection(name)
        c = cls(collection_name=name, embedding_size=32, device="cpu")
        c.update(docs, emb.tolist(), name)
        text, sources = c.search(emb[17].tolist(), limit=3)
        assert text.startswith(f"[[DOCUMENT {first}]]\n\ncontent 17\n\n")
        assert "file17.pdf" in sources and sources["file17.pdf"]["doc_metadata"]["page_num"] == 17
        assert len(sources) == 3
    q = QdrantStyleClient(collection_name="test_QdrantStyleClient", embedding_size=32, device="cpu")
    q.update(docs[:10], emb[:10].tolist(), "test_QdrantStyleClient")  # upsert: same ids replaced
    assert len(q._col().index) == 300
    m = MilvusStyleClient(collection_name="test_MilvusStyleClient", embedding_size=32, device="cpu")
    m.update(docs[:10], emb[:10].tolist(), "test_MilvusStyleClient")  # insert: appended
    assert len(m._col().payloads) == 310


def test_tracing_callback_spans_first_token_and_retry():
    """TracingCallback (the reference's OpenTelemetryCallbackHandler, C19/C20): nested spans
    by run id, first-token latency, token counts, retriever documents, tool spans, retries,
    process metrics at span end."""
    import time as _t

    from nv_genai_amd.observability.tracing import InMemoryExporter, Tracer, TracingCallback

    exp = InMemoryExporter()
    cb = TracingCallback(Tracer("chain-server", exp, enabled=True), token_events=True)
    cb.on_chain_start("c1", "rag_chain", inputs={"q": "capital?"})
    cb.on_retriever_start("r1", "capital?", parent_run_id="c1")
    cb.on_retriever_end("r1", [("Quartz City doc", 0.9)])
    cb.on_llm_start("l1", ["prompt"], parent_run_id="c1", temperature=0.2)
    _t.sleep(0.002)
    for tok in ("Quartz", " City"):
        cb.on_llm_new_token("l1", tok)
    cb.on_retry("l1", 1, "timeout")
    cb.on_llm_end("l1", "Quartz City", prompt_tokens=12)
    cb.on_tool_start("t1", "Math", "2+2", parent_run_id="c1")
    cb.on_tool_end("t1", "4")
    cb.on_chain_end("c1", outputs="Quartz City")
    by = {s.name: s for s in exp.spans}
    assert set(by) == {"rag_chain", "retriever", "llm", "tool:Math"}
    for n in ("retriever", "llm", "tool:Math"):
        assert by[n].parent_id == by["rag_chain"].span_id and by[n].trace_id == by["rag_chain"].trace_id
    llm = by["llm"].attributes
    assert llm["completion_tokens"] == 2 and llm["prompt_tokens"] == 12 and llm["first_token_time_ms"] >= 1.0
    assert by["retriever"].attributes["documents.0.score"] == 0.9
    names = [e["name"] for e in by["llm"].events]
    assert names.count("new_token") == 2 and "retry" in names
