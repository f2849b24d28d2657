"""Streaming ingest pipeline on CPU: file/RSS/custom sources, chunking, batched embedding,
routing to named stores, the isolate-embeddings trigger and back-pressure."""
import os
import threading

import pytest

from nv_genai_amd.connectors.fake import HashEmbeddings
from nv_genai_amd.index.vectorstore import VectorStore
from nv_genai_amd.ingest.streaming import IngestPipeline, parse_feed

RSS = """<?xml version="1.0"?><rss version="2.0"><channel><title>sec</title>
<item><title>Patch Tuesday</title><link>https://example.org/a</link><description>Fixes for 60 flaws including a zero day in the kernel.</description></item>
<item><title>Botnet</title><link>https://example.org/b</link><description>A new botnet targets routers.</description></item>
</channel></rss>"""
ATOM = """<?xml version="1.0" encoding="utf-8"?><feed xmlns="http://www.w3.org/2005/Atom"><title>t</title>
<entry><title>Atom one</title><link href="https://example.org/c"/><summary>short</summary><content>long content body of the entry</content></entry>
</feed>"""


class Emb(HashEmbeddings):
    def __init__(self):
        super().__init__(dim=64)
        self.calls = []

    def embed(self, texts, input_type="passage", truncate="END"):
        self.calls.append(len(texts))
        return super().embed(texts, input_type, truncate)


def _factory(stores):
    def make(name, recreate):
        st = VectorStore(HashEmbeddings(dim=64), 64, device="cpu", name=name)
        stores[name] = st
        return st
    return make


def test_parse_feeds():
    r = parse_feed(RSS)
    assert [e["title"] for e in r] == ["Patch Tuesday", "Botnet"] and r[0]["link"] == "https://example.org/a"
    a = parse_feed(ATOM)
    assert a[0]["link"] == "https://example.org/c" and a[0]["content"].startswith("long content")


def test_file_rss_custom_sources_to_named_stores(tmp_path):
    for i in range(3):
        (tmp_path / f"doc{i}.txt").write_text(("security advisory paragraph %d. " % i) * 80)
    (tmp_path / "feed.xml").write_text(RSS)
    (tmp_path / "logs.csv").write_text("raw,request_header_referer,other\nGET /a,ref1,x\nPOST /b,ref2,y\n")
    cfg = {"vdb_pipeline": {
        "pipeline": {"edge_buffer_size": 4, "max_batch_size": 16, "num_threads": 2, "pipeline_batch_size": 8,
                     "chunk_size": 256},
        "vdb": {"batch_size": 10, "resource_name": "VDBGENERAL"},
        "sources": [
            {"type": "filesystem", "name": "txt", "config": {"filenames": [str(tmp_path / "*.txt")],
                                                             "vdb_resource_name": "vdb_pdf"}},
            {"type": "filesystem", "name": "csv", "config": {
                "filenames": [str(tmp_path / "logs.csv")], "vdb_resource_name": "vdb_csv",
                "converters_meta": {"csv": {"text_column_names": ["raw", "request_header_referer"]}}}},
            {"type": "rss", "name": "rss", "config": {"feed_input": [str(tmp_path / "feed.xml")],
                                                      "vdb_resource_name": "vdb_rss"}},
            {"type": "custom", "name": "custom", "config": {}},
        ]}}
    emb, stores = Emb(), {}
    p = IngestPipeline(cfg, emb, _factory(stores))
    custom = p.sources[-1]
    custom.push({"payload": "pushed at runtime about ransomware", "source": "producer"})
    custom.push(None)
    mons = p.run(timeout=30)
    assert not p.errors
    assert set(stores) == {"vdb_pdf", "vdb_csv", "vdb_rss", "VDBGENERAL"}
    assert len(stores["vdb_csv"]) == 2 and len(stores["vdb_rss"]) == 2 and len(stores["VDBGENERAL"]) == 1
    assert len(stores["vdb_pdf"]) >= 3 * 9                      # ~2.6 KB docs / 256-char chunks
    assert max(emb.calls) <= 16                                   # micro-batched to max_batch_size
    assert mons["upload"].count == sum(len(s) for s in stores.values())
    hit = stores["vdb_csv"].similarity_search("GET /a ref1", 1)[0]
    assert hit.page_content == "GET /a ref1" and hit.metadata["source"].endswith("logs.csv")


def test_isolate_embeddings_trigger(tmp_path):
    (tmp_path / "a.txt").write_text("alpha " * 400)
    cfg = {"vdb_pipeline": {"embeddings": {"isolate_embeddings": True},
                            "pipeline": {"max_batch_size": 1000, "chunk_size": 128},
                            "sources": [{"type": "filesystem", "config": {"filenames": [str(tmp_path / "a.txt")]}}]}}
    emb, stores = Emb(), {}
    IngestPipeline(cfg, emb, _factory(stores)).run(timeout=30)
    assert len(emb.calls) == 1                       # everything held until the sources finished


def test_kafka_source_refuses_without_client():
    cfg = {"vdb_pipeline": {"sources": [{"type": "kafka", "name": "k", "config": {}}]}}
    p = IngestPipeline(cfg, Emb(), _factory({}))
    p.run(timeout=10)
    assert p.errors and "kafka" in p.errors[0]


def test_pipeline_without_timeout_and_rate_benchmark(tmp_path):
    """run(timeout=None) waits for finite sources (the CLI default); the ingest-rate benchmark
    indexes every chunk it produced."""
    import json
    import os
    import subprocess
    import sys

    out = tmp_path / "ing.json"
    r = subprocess.run([sys.executable, "benchmarks/ingest_rate.py", "--docs", "30", "--embed-model", "encoder-tiny",
                        "--threads", "2", "--out", str(out)], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=os.getcwd()))
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(out.read_text())
    assert res["chunks"] > 30 and res["indexed"] == res["chunks"] and res["value"] > 0
