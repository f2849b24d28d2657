"""Streaming document ingest: sources → chunker → embedder → vector-DB writer, as a
pipeline of stages connected by bounded queues (reference:
experimental/streaming_ingest_rag/morpheus_examples/streaming_ingest_rag/vdb_upload/
{pipeline.py:29-110, vdb_config.yaml, module/*.py}, a Morpheus/MRC pipeline feeding Triton
and Milvus).

* sources (``vdb_pipeline.sources``): ``filesystem`` (glob list, optional ``watch``; text/
  PDF/HTML/CSV through the loaders, CSV rows → concatenated ``text_column_names``), ``rss``
  (RSS 2.0 / Atom feeds from URLs or files, entries optionally scraped with the web scraper,
  an HTTP response cache, ``interval_sec`` polling or one shot), ``kafka`` (needs a Kafka
  client library; absent here, so the stage refuses loudly), ``custom`` (an in-process queue
  any producer can push raw text or URLs into);
* ``raw_chunk``: recursive character splitting (native ``_rt.char_split``), chunk_size with
  chunk_size // 10 overlap, one output row per chunk carrying the source metadata;
* embedding: micro-batches of ``max_batch_size`` chunks through the in-process GPU encoder
  (the Triton ``all-MiniLM-L6-v2`` role: ``PreprocessNLPStage`` + ``TritonInferenceStage``);
* ``WriteToVectorDBStage``: rows are routed by ``vdb_resource_name`` to named in-HBM vector
  stores and flushed in ``vdb.batch_size`` groups (``recreate`` honoured);
* ``MonitorStage`` rates (chunks/s, embeddings/s, uploads/s) and an optional ``TriggerStage``
  (``isolate_embeddings``: hold everything until the sources finish, to time the GPU stage
  on its own).

Stages run on their own threads (``pipeline.num_threads`` workers for the chunker), so
source I/O, chunking, GPU inference and index writes overlap (pipeline parallelism); the
queues are ``edge_buffer_size`` deep, so a slow stage back-pressures its producers.
"""
from __future__ import annotations

import csv
import glob
import hashlib
import json
import logging
import os
import queue
import threading
import time
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field
from typing import Callable, Dict, Iterable, Iterator, List, Optional

log = logging.getLogger(__name__)
_END = object()


@dataclass
class Row:
    content: str
    source: str = ""
    title: str = ""
    summary: str = ""
    resource: str = "VDBGENERAL"
    meta: Dict = field(default_factory=dict)


class Monitor:
    def __init__(self, name: str, unit: str):
        self.name, self.unit, self.count, self.t0 = name, unit, 0, None
        self.lock = threading.Lock()

    def add(self, n: int):
        with self.lock:
            if self.t0 is None:
                self.t0 = time.perf_counter()
            self.count += n

    def rate(self) -> float:
        if self.t0 is None:
            return 0.0
        return self.count / max(1e-9, time.perf_counter() - self.t0)

    def __repr__(self):
        return f"{self.name}: {self.count} {self.unit} ({self.rate():.1f} {self.unit}/s)"


# ---------------------------------------------------------------------------- sources
class Source:
    name = "source"

    def __init__(self, cfg: dict, resource: str):
        self.cfg, self.resource = cfg, resource

    def rows(self, stop: threading.Event) -> Iterator[Row]:
        raise NotImplementedError


class FileSource(Source):
    name = "filesystem"

    def _read(self, path: str) -> Iterator[Row]:
        meta = (self.cfg.get("converters_meta") or {})
        if path.lower().endswith(".csv"):
            cols = (meta.get("csv") or {}).get("text_column_names") or []
            with open(path, newline="", encoding="utf-8", errors="replace") as f:
                for r in csv.DictReader(f):
                    text = " ".join(str(r.get(c, "")) for c in cols) if cols else " ".join(map(str, r.values()))
                    yield Row(text, source=path, title=os.path.basename(path), resource=self.resource)
            return
        from ..rag.loaders import load_file

        for d in load_file(path):
            yield Row(d.page_content, source=path, title=os.path.basename(path), resource=self.resource,
                      meta=dict(d.metadata))

    def rows(self, stop):
        seen = set()
        while not stop.is_set():
            for pat in self.cfg.get("filenames", []):
                for path in sorted(glob.glob(pat)):
                    if path in seen:
                        continue
                    seen.add(path)
                    try:
                        yield from self._read(path)
                    except Exception as e:  # noqa: BLE001 - one bad file must not stop ingest
                        log.error("failed to read %s: %s", path, e)
            if not self.cfg.get("watch", False):
                return
            stop.wait(float(self.cfg.get("watch_interval", 1.0)))


def _text(el: Optional[ET.Element]) -> str:
    return "".join(el.itertext()).strip() if el is not None else ""


def parse_feed(xml_text: str) -> List[dict]:
    """RSS 2.0 items or Atom entries → [{"title", "link", "summary", "content"}]."""
    root = ET.fromstring(xml_text)
    ns = {"a": "http://www.w3.org/2005/Atom"}
    out = []
    for it in root.iter("item"):
        out.append({"title": _text(it.find("title")), "link": _text(it.find("link")),
                    "summary": _text(it.find("description")), "content": ""})
    for e in root.findall(".//a:entry", ns):
        link = e.find("a:link", ns)
        out.append({"title": _text(e.find("a:title", ns)), "link": link.get("href", "") if link is not None else "",
                    "summary": _text(e.find("a:summary", ns)), "content": _text(e.find("a:content", ns))})
    return out


class HTTPCache:
    """Response cache keyed on the URL (the reference's requests_cache SQLite role)."""

    def __init__(self, cache_dir: Optional[str]):
        self.dir = cache_dir
        if cache_dir:
            os.makedirs(cache_dir, exist_ok=True)

    def get(self, url: str, timeout: float) -> str:
        if self.dir:
            p = os.path.join(self.dir, hashlib.sha256(url.encode()).hexdigest())
            if os.path.exists(p):
                with open(p, encoding="utf-8") as f:
                    return f.read()
        if url.startswith(("http://", "https://")):
            import requests

            r = requests.get(url, timeout=timeout)
            r.raise_for_status()
            text = r.text
        else:
            with open(url.replace("file://", ""), encoding="utf-8") as f:
                text = f.read()
        if self.dir:
            with open(p, "w", encoding="utf-8") as f:
                f.write(text)
        return text


def scrape(html: str) -> str:
    from ..rag.loaders import html_to_text

    return html_to_text(html)


class RSSSource(Source):
    name = "rss"

    def rows(self, stop):
        cache = HTTPCache(self.cfg.get("cache_dir") if self.cfg.get("enable_cache") else None)
        timeout = float(self.cfg.get("request_timeout_sec", 2.0))
        scrape_cfg = self.cfg.get("web_scraper_config")
        seen = set()
        t_end = time.time() + float(self.cfg.get("stop_after_sec", 0) or 1e18)
        while not stop.is_set() and time.time() < t_end:
            for feed in self.cfg.get("feed_input", []):
                try:
                    entries = parse_feed(cache.get(feed, timeout))
                except Exception as e:  # noqa: BLE001
                    log.warning("feed %s failed: %s", feed, e)
                    continue
                for en in entries:
                    key = en["link"] or en["title"]
                    if key in seen:
                        continue
                    seen.add(key)
                    text = en["content"] or en["summary"]
                    if scrape_cfg is not None and en["link"]:
                        try:
                            text = scrape(cache.get(en["link"], timeout)) or text
                        except Exception as e:  # noqa: BLE001
                            log.debug("scrape of %s failed: %s", en["link"], e)
                    yield Row(text, source=en["link"] or feed, title=en["title"], summary=en["summary"],
                              resource=self.resource)
            if not self.cfg.get("run_indefinitely", False):
                return
            stop.wait(float(self.cfg.get("interval_sec", 600)))


class KafkaSource(Source):
    name = "kafka"

    def rows(self, stop):
        try:
            from kafka import KafkaConsumer  # type: ignore
        except ImportError as e:
            raise RuntimeError("the kafka source needs the kafka-python package, which is not installed") from e
        c = KafkaConsumer(*self.cfg.get("topics", ["raw_queue"]), bootstrap_servers=self.cfg.get("bootstrap_servers"),
                          group_id=self.cfg.get("group_id", "vdb_upload"), consumer_timeout_ms=1000)
        while not stop.is_set():
            for msg in c:
                d = json.loads(msg.value)
                yield Row(d.get("payload", d.get("content", "")), source=d.get("source", "kafka"),
                          title=d.get("title", ""), resource=self.resource)


class CustomSource(Source):
    """In-process producer queue: push dicts {"payload" | "content" | "url", ...}; ``None`` ends."""

    name = "custom"

    def __init__(self, cfg, resource):
        super().__init__(cfg, resource)
        self.q: "queue.Queue" = queue.Queue()

    def push(self, item: Optional[dict]):
        self.q.put(item)

    def rows(self, stop):
        while not stop.is_set():
            try:
                d = self.q.get(timeout=0.1)
            except queue.Empty:
                continue
            if d is None:
                return
            text = d.get("payload") or d.get("content") or ""
            if not text and d.get("url"):
                text = scrape(HTTPCache(None).get(d["url"], 5.0))
            yield Row(text, source=d.get("source", d.get("url", "custom")), title=d.get("title", ""),
                      resource=self.resource)


SOURCES = {"filesystem": FileSource, "rss": RSSSource, "kafka": KafkaSource, "custom": CustomSource}


# ---------------------------------------------------------------------------- pipeline
class IngestPipeline:
    def __init__(self, config: dict, embedder, store_factory: Callable[[str, int], object]):
        vp = config.get("vdb_pipeline", config)
        self.pcfg = vp.get("pipeline", {})
        self.vcfg = vp.get("vdb", {})
        self.ecfg = vp.get("embeddings", {})
        self.embedder = embedder
        self.store_factory = store_factory
        self.stores: Dict[str, object] = {}
        depth = int(self.pcfg.get("edge_buffer_size", 128))
        self.q_src: "queue.Queue" = queue.Queue(depth)
        self.q_chunk: "queue.Queue" = queue.Queue(depth)
        self.q_emb: "queue.Queue" = queue.Queue(depth)
        self.stop = threading.Event()
        self.sources: List[Source] = []
        for s in vp.get("sources", []):
            c = s.get("config", {})
            cls = SOURCES[s["type"]]
            self.sources.append(cls(c, c.get("vdb_resource_name", self.vcfg.get("resource_name", "VDBGENERAL"))))
            self.sources[-1].name = s.get("name", s["type"])
        self.monitors = {"source": Monitor("Source rate", "rows"), "chunk": Monitor("Chunk rate", "chunks"),
                         "embed": Monitor("Inference rate", "embeddings"), "upload": Monitor("Upload rate", "embeddings")}
        self.errors: List[str] = []

    # -- stage bodies
    def _run_source(self, src: Source):
        try:
            for row in src.rows(self.stop):
                self.q_src.put(row)
                self.monitors["source"].add(1)
        except Exception as e:  # noqa: BLE001
            self.errors.append(f"{src.name}: {e}")
            log.error("source %s failed: %s", src.name, e)

    def _chunker(self):
        from ..rag.splitters import RecursiveCharacterTextSplitter

        size = int(self.pcfg.get("chunk_size", 512))
        sp = RecursiveCharacterTextSplitter(size, int(self.pcfg.get("chunk_overlap", size // 10)))
        batch, n = [], int(self.pcfg.get("pipeline_batch_size", 128))
        while True:
            row = self.q_src.get()
            if row is _END:
                break
            for piece in sp.split_text(row.content):
                batch.append(Row(piece, row.source, row.title, row.summary, row.resource, row.meta))
            if len(batch) >= n:
                self.q_chunk.put(batch)
                self.monitors["chunk"].add(len(batch))
                batch = []
        if batch:
            self.q_chunk.put(batch)
            self.monitors["chunk"].add(len(batch))

    def _embed(self):
        mb = int(self.pcfg.get("max_batch_size", 256))
        buf: List[Row] = []
        held: List[List[Row]] = []
        isolate = bool(self.ecfg.get("isolate_embeddings", False))
        done = False
        while not done:
            item = self.q_chunk.get()
            if item is _END:
                done = True
            elif isolate:
                held.append(item)         # TriggerStage: release only after the sources finish
                continue
            else:
                buf.extend(item)
            if done and isolate:
                for h in held:
                    buf.extend(h)
            while len(buf) >= mb or (done and buf):
                part, buf = buf[:mb], buf[mb:]
                vecs = self.embedder.embed([r.content for r in part], input_type="passage")
                self.q_emb.put((part, vecs))
                self.monitors["embed"].add(len(part))

    def _store(self, name: str):
        if name not in self.stores:
            self.stores[name] = self.store_factory(name, bool(self.vcfg.get("recreate", True)))
        return self.stores[name]

    def _writer(self):
        bs = int(self.vcfg.get("batch_size", 5120))
        pend: Dict[str, list] = {}

        def flush(name):
            rows, vecs = zip(*pend.pop(name))
            import torch

            st = self._store(name)
            st.add_texts([r.content for r in rows],
                         [{"source": r.source, "title": r.title, "summary": r.summary, **r.meta} for r in rows],
                         embeddings=torch.stack(list(vecs)))
            self.monitors["upload"].add(len(rows))

        while True:
            item = self.q_emb.get()
            if item is _END:
                break
            rows, vecs = item
            for r, v in zip(rows, vecs):
                pend.setdefault(r.resource, []).append((r, v))
                if len(pend[r.resource]) >= bs:
                    flush(r.resource)
        for name in list(pend):
            flush(name)

    def run(self, timeout: Optional[float] = None) -> Dict[str, Monitor]:
        """Run until every (finite) source is exhausted and all stages drained."""
        nthreads = max(1, int(self.pcfg.get("num_threads", 1)))
        srcs = [threading.Thread(target=self._run_source, args=(s,), daemon=True) for s in self.sources]
        chunkers = [threading.Thread(target=self._chunker, daemon=True) for _ in range(nthreads)]
        emb = threading.Thread(target=self._embed, daemon=True)
        wr = threading.Thread(target=self._writer, daemon=True)
        for t in srcs + chunkers + [emb, wr]:
            t.start()
        t_end = None if timeout is None else time.time() + timeout
        for t in srcs:
            t.join(None if t_end is None else max(0.0, t_end - time.time()))
        self.stop.set()
        for _ in chunkers:
            self.q_src.put(_END)
        for t in chunkers:
            t.join()
        self.q_chunk.put(_END)
        emb.join()
        self.q_emb.put(_END)
        wr.join()
        for m in self.monitors.values():
            log.info("%s", m)
        return self.monitors


def load_config(path: str) -> dict:
    import yaml

    with open(path) as f:
        return yaml.safe_load(f)


def store_kwargs(vcfg: dict, name: str) -> dict:
    """VectorStore arguments for a collection from the reference's vdb ``resource_schemas``
    ``index_conf`` (kafka_config.yaml:109-125: ``metric_type`` L2 / IP / COSINE, ``index_type``
    HNSW with ``M`` / ``efConstruction``, or IVF_FLAT / GPU_IVF_FLAT with ``nlist``; anything
    else is the flat in-HBM scan)."""
    conf = ((vcfg.get("resource_schemas") or {}).get(name) or {}).get("index_conf") or {}
    if not conf:
        return {}
    params = conf.get("params") or {}
    out = {"metric": {"L2": "l2", "IP": "ip", "COSINE": "cosine"}.get(str(conf.get("metric_type", "")).upper(),
                                                                        "cosine")}
    it = str(conf.get("index_type", "")).upper()
    if it == "HNSW":
        out.update(index_type="hnsw", hnsw_m=int(params.get("M", 16)),
                   hnsw_ef_construction=int(params.get("efConstruction", 200)))
    elif it in ("IVF_FLAT", "GPU_IVF_FLAT"):
        out.update(index_type="ivf_flat", nlist=int(params.get("nlist", 64)))
    else:
        out["index_type"] = "flat"
    return out


def main(argv=None):
    import argparse

    ap = argparse.ArgumentParser(description="Streaming ingest into the in-HBM vector stores")
    ap.add_argument("--config", required=True, help="vdb_pipeline YAML (reference vdb_config.yaml layout)")
    ap.add_argument("--embed-model", default="all-minilm-l6-v2")
    ap.add_argument("--persist-dir", default=None)
    ap.add_argument("--timeout", type=float, default=None)
    a = ap.parse_args(argv)
    from ..engine.embed_engine import EmbeddingEngine
    from ..index.vectorstore import VectorStore

    emb = EmbeddingEngine(a.embed_model)
    cfg = load_config(a.config)
    vcfg = cfg.get("vdb_pipeline", cfg).get("vdb", {}) if isinstance(cfg, dict) else {}

    def factory(name, recreate):
        return VectorStore(emb, emb.dim, name=name,
                           persist_dir=os.path.join(a.persist_dir, name) if a.persist_dir else None,
                           **store_kwargs(vcfg, name))

    mons = IngestPipeline(cfg, emb, factory).run(a.timeout)
    for m in mons.values():
        print(m)


if __name__ == "__main__":
    main()
