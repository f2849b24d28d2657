"""Factories shared by the example chains (RetrievalAugmentedGeneration/common/utils.py:100-468).

Backends are picked from the ``AppConfig``:

* ``llm.model_engine``: ``local`` (in-process Llama engine on this GPU, hipGraph decode),
  ``nvidia-ai-endpoints`` / ``openai`` (OpenAI/NIM HTTP protocol at ``llm.server_url`` —
  e.g. this framework's model server), ``fake`` (deterministic test model);
* ``embeddings.model_engine``: ``local`` (in-process encoder), ``nvidia-ai-endpoints`` /
  ``openai`` (HTTP ``/v1/embeddings``), ``hash`` (feature-hashing test embedder);
* vector store: always the in-HBM index of this framework; ``vector_store.name`` milvus /
  pgvector / faiss are accepted for compatibility, ``index.type`` flat | ivf_flat picks the
  structure, ``index.persist_dir`` enables snapshots, ``COLLECTION_NAME`` names the collection.

Quirk kept on purpose: only temperature / top_p / max_tokens of the request reach the LLM
(``stop`` is accepted by the API but dropped — utils.py:271-286).
"""
from __future__ import annotations

import logging
import os
import threading
from functools import lru_cache
from typing import Any, Dict, List, Optional

from .configuration import AppConfig

log = logging.getLogger(__name__)
DEFAULT_MAX_CONTEXT = 1500
_LOCK = threading.RLock()
_RUNTIME: Dict[str, Any] = {}


@lru_cache(maxsize=1)
def get_config() -> AppConfig:
    path = os.environ.get("APP_CONFIG_FILE", "/dev/null")
    cfg = AppConfig.from_file(path) if path != "/dev/null" else None
    return cfg if cfg is not None else AppConfig.from_dict({})


def reset():
    """Drop cached config / engines / stores (tests)."""
    from ..index.vectorstore import reset_stores

    get_config.cache_clear()
    with _LOCK:
        svc = _RUNTIME.get("llm_service")
        if svc is not None:
            svc.shutdown()
        _RUNTIME.clear()
    reset_stores()


def _device(cfg: AppConfig) -> str:
    import torch

    return cfg.engine.device or ("cuda" if torch.cuda.is_available() else "cpu")


def register_runtime(name: str, obj) -> None:
    """Inject a pre-built engine/service (e.g. the model server shares its engines)."""
    with _LOCK:
        _RUNTIME[name] = obj


def get_llm_service():
    with _LOCK:
        svc = _RUNTIME.get("llm_service")
        if svc is None:
            from ..engine.llm_engine import EngineConfig, LLMEngine
            from ..serving.engine_service import EngineService

            cfg = get_config()
            e = cfg.engine
            weights = None
            if e.weights_dir:
                from ..utils.checkpoint import load_weights

                weights = load_weights(e.weights_dir)
            eng = LLMEngine(EngineConfig(model=e.llm_preset, max_num_seqs=e.max_num_seqs,
                                         max_model_len=e.max_model_len,
                                         max_batched_tokens=e.max_batched_tokens,
                                         kv_cache_fraction=e.kv_cache_fraction,
                                         kv_cache_dtype=e.kv_cache_dtype, fp8=e.fp8),
                            device=_device(cfg), weights=weights)
            svc = EngineService(eng)
            _RUNTIME["llm_service"] = svc
        return svc


def get_embedding_engine():
    with _LOCK:
        eng = _RUNTIME.get("embed_engine")
        if eng is None:
            from ..engine.embed_engine import EmbeddingEngine

            cfg = get_config()
            eng = EmbeddingEngine(cfg.engine.embed_preset, device=_device(cfg))
            _RUNTIME["embed_engine"] = eng
        return eng


def get_rerank_engine():
    with _LOCK:
        eng = _RUNTIME.get("rerank_engine")
        cfg = get_config()
        if eng is None and cfg.engine.rerank_preset:
            from ..engine.embed_engine import EmbeddingEngine

            eng = EmbeddingEngine(cfg.engine.rerank_preset, device=_device(cfg))
            _RUNTIME["rerank_engine"] = eng
        return eng


def get_llm(**kwargs):
    """Chat model for the configured backend; forwards temperature/top_p/max_tokens only."""
    cfg = get_config()
    settings = {k: kwargs[k] for k in ("temperature", "top_p", "max_tokens") if kwargs.get(k) is not None}
    engine = cfg.llm.model_engine
    if engine == "fake":
        from ..connectors.fake import FakeChatModel

        fake = _RUNTIME.get("fake_llm")
        return fake if fake is not None else FakeChatModel(**settings)
    if engine == "local":
        from ..connectors.local import LocalChatModel

        return LocalChatModel(get_llm_service(), cfg.llm.model_name, **settings)
    if engine in ("nvidia-ai-endpoints", "openai", "nim"):
        from ..connectors.http import ChatClient

        url = cfg.llm.server_url or "https://integrate.api.nvidia.com/v1"
        return ChatClient(url, cfg.llm.model_name, **settings)
    raise RuntimeError(f"Unsupported llm model engine: {engine}")


def get_embedding_model():
    cfg = get_config()
    engine = cfg.embeddings.model_engine
    if engine in ("hash", "fake"):
        from ..connectors.fake import HashEmbeddings

        return HashEmbeddings(cfg.embeddings.dimensions)
    if engine in ("local", "huggingface"):
        from ..connectors.local import LocalEmbeddings

        return LocalEmbeddings(get_embedding_engine(), cfg.embeddings.model_name)
    if engine in ("nvidia-ai-endpoints", "openai", "nim"):
        from ..connectors.http import EmbeddingsClient

        url = cfg.embeddings.server_url or "https://integrate.api.nvidia.com/v1"
        return EmbeddingsClient(url, cfg.embeddings.model_name, truncate="END")
    raise RuntimeError(f"Unsupported embedding model engine: {engine}")


def get_reranker(top_n: int = 4):
    cfg = get_config()
    eng = get_rerank_engine()
    if eng is not None:
        from ..connectors.local import LocalReranker

        return LocalReranker(eng, cfg.engine.rerank_preset, top_n)
    if cfg.retriever.nr_url and cfg.llm.model_engine not in ("local", "fake"):
        from ..connectors.http import RerankClient

        return RerankClient(cfg.retriever.nr_url, top_n=top_n)
    return None


def collection_name(default: str = "default") -> str:
    return os.environ.get("COLLECTION_NAME", default) or default


def get_vectorstore(collection: Optional[str] = None):
    """Named in-HBM vector store (created on first use, snapshot-backed if configured)."""
    from ..index.vectorstore import VectorStore, get_store

    cfg = get_config()
    name = collection or collection_name()

    def make(n):
        emb = get_embedding_model()
        dim = getattr(emb, "dim", cfg.embeddings.dimensions)
        persist = os.path.join(cfg.index.persist_dir, n) if cfg.index.persist_dir else None
        itype = cfg.index.type
        if cfg.vector_store.name == "milvus" and itype == "flat" and os.environ.get("APP_INDEX_TYPE") is None:
            itype = "flat"  # GPU brute force beats IVF at these sizes; set APP_INDEX_TYPE=ivf_flat for IVF
        dev = _device(cfg) if cfg.embeddings.model_engine not in ("hash", "fake") else "cpu"
        vs = VectorStore(emb, dim, itype, cfg.index.metric, dev, cfg.vector_store.nlist,
                         cfg.vector_store.nprobe, name=n, persist_dir=persist)
        if cfg.index.synthetic_docs and n == collection_name() and len(vs) == 0:
            _fill_synthetic(vs, cfg)
        return vs

    return get_store(name, make)


def _fill_synthetic(vs, cfg) -> None:
    """Benchmark corpus for the REST path (the same synthetic data as bench.py): random unit
    vectors + generated ~500-token chunks, and a whitened query encoder so concurrent
    questions retrieve different chunks (a random-init encoder's outputs are nearly collinear)."""
    from ..index.docstore import SyntheticDocStore
    from ..utils.synthetic import TextGen

    n = int(cfg.index.synthetic_docs)
    vs.index.add_random(n, seed=1234)
    vs.docs = SyntheticDocStore(n)
    vs._mark_write()
    cal = TextGen(seed=999)
    questions = [cal.question() for _ in range(4096)]
    if cfg.embeddings.model_engine in ("local", "huggingface"):
        get_embedding_engine().calibrate_whitening(questions)
    elif hasattr(vs.embedder, "embed_query_tensor"):
        # the encoder sits behind HTTP (a model server, the reference's NIM topology): whiten
        # its query vectors here, from the same calibration questions, so the split topology
        # retrieves as diversely as the in-process one (unwhitened random-init vectors are
        # nearly collinear: every question would retrieve the same chunks and hit the prefix
        # cache on the whole prompt)
        from ..engine.embed_engine import pca_whitening
        from ..index.vectorstore import WhitenedEmbedder

        mu, W = pca_whitening(vs.embedder.embed_query_tensor(questions))
        vs.embedder = WhitenedEmbedder(vs.embedder, mu, W, device=vs.index_device())
    log.info("filled collection %s with %d synthetic chunks", vs.name, n)


create_vectorstore_langchain = get_vectorstore


def get_text_splitter():
    from ..rag.splitters import TokenTextSplitter

    cfg = get_config()
    return TokenTextSplitter(tokens_per_chunk=cfg.text_splitter.chunk_size - 2,
                             chunk_overlap=cfg.text_splitter.chunk_overlap)


def get_docs_vectorstore(vs) -> List[str]:
    return vs.get_filenames()


def del_docs_vectorstore(vs, filenames: List[str]) -> bool:
    """Delete every chunk of each filename. Kept quirk: like the Milvus path of the reference
    (utils.py:400,465) this returns after the first filename that was found."""
    for f in filenames:
        if vs.delete_by_filename(f):
            return True
    return False


def llm_tokenizer_len(text: str) -> int:
    from ..utils.tokenizer import llm_tokenizer

    return len(llm_tokenizer().encode(text))


class LimitRetrievedNodesLength:
    """Keep retrieved documents in rank order until the running token count exceeds
    DEFAULT_MAX_CONTEXT (utils.py:97-122)."""

    def __init__(self, limit: int = DEFAULT_MAX_CONTEXT, count=None):
        self.limit = limit
        self.count = count

    def postprocess(self, docs):
        texts = [d.page_content if hasattr(d, "page_content") else d[0].page_content for d in docs]
        if self.count is None:
            # one batched encode (the Rust tokenizer runs it without the GIL) instead of a
            # GIL-holding encode per document on every request's worker thread
            from ..utils.tokenizer import llm_tokenizer

            counts = [len(ids) for ids in llm_tokenizer().encode_batch(texts)] if texts else []
        else:
            counts = [self.count(t) for t in texts]
        out, total = [], 0
        for d, n in zip(docs, counts):
            total += n
            if total > self.limit:
                break
            out.append(d)
        return out
