"""In-process RAG serving pipeline: embed -> vector search -> context cap -> prompt -> LLM.

This is the canonical QA chain of the reference (``developer_rag``,
RetrievalAugmentedGeneration/examples/developer_rag/chains.py:141-176) with the service hops
removed: instead of HTTP to an embedding microservice, gRPC to Milvus and HTTP to NIM, the
three engines share one process per GPU and hand tensors to each other in HBM.

Semantics kept from the reference:
* top_k = 4 retrieval (configuration.py:141-145);
* ``LimitRetrievedNodesLength``: nodes are taken in rank order until the running token count
  would exceed 1500, then dropped (utils.py:97-122);
* the ``rag_template`` prompt (configuration.py:180-189) sent as a user chat message, so the
  model server renders it with the Llama-3 chat template.

Prompts are assembled in token space: the template's fixed parts and every chunk's token ids
are tokenised once (chunk ids are cached in the docstore at ingest), only the question is
tokenised per request.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import torch

from ..engine.embed_engine import EmbeddingEngine
from ..engine.llm_engine import LLMEngine, Request, SamplingParams
from ..index.docstore import DocStore

RAG_TEMPLATE = (
    "<s>[INST] <<SYS>>"
    "Use the following context to answer the user's question. If you don't know the answer,"
    "just say that you don't know, don't try to make up an answer."
    "<</SYS>>"
    "<s>[INST] Context: {context_str} Question: {query_str} Only return the helpful"
    " answer below and nothing else. Helpful answer:[/INST]"
)
DEFAULT_MAX_CONTEXT = 1500


@dataclass
class RAGResult:
    question: str
    request: Request
    doc_ids: List[int]
    scores: List[float]
    t_start: float
    t_retrieved: float
    prompt_tokens: int

    @property
    def answer(self) -> str:
        return self.request.text

    @property
    def ttft(self) -> Optional[float]:
        ft = self.request.first_token_time
        return None if ft is None else ft - self.t_start

    @property
    def latency(self) -> Optional[float]:
        ft = self.request.finish_time
        return None if ft is None else ft - self.t_start


@dataclass
class PendingRetrieval:
    questions: List[str]
    params: SamplingParams
    scores: torch.Tensor
    ids: torch.Tensor
    event: Optional["torch.cuda.Event"]
    t0: float
    keep: tuple = ()     # device tensors kept alive until the copies complete


class RAGPipeline:
    def __init__(self, llm: LLMEngine, embedder: EmbeddingEngine, index, docstore: DocStore,
                 top_k: int = 4, max_context_tokens: int = DEFAULT_MAX_CONTEXT,
                 template: str = RAG_TEMPLATE, score_threshold: Optional[float] = None):
        self.llm, self.embedder, self.index, self.docs = llm, embedder, index, docstore
        self.top_k = top_k
        self.max_ctx = max_context_tokens
        self.score_threshold = score_threshold
        self.set_template(template)
        # retrieval runs on its own HIP stream so query embedding + search of newly arriving
        # requests overlap the LLM step in flight instead of queueing behind it
        dev = getattr(embedder, "device", torch.device("cpu"))
        self.stream = torch.cuda.Stream(dev) if torch.device(dev).type == "cuda" else None
        # host seconds spent in each part of submit_async (bench.py reports them)
        self.submit_host_s = {"tokenize": 0.0, "embed": 0.0, "search": 0.0, "copy": 0.0}

    def set_template(self, template: str):
        tok = self.llm.tok
        pre, rest = template.split("{context_str}", 1)
        mid, post = rest.split("{query_str}", 1)
        hdr = [tok.bos_id, tok.header_start] + tok.encode("user") + [tok.header_end] + tok.encode("\n\n")
        self._pre = hdr + tok.encode(pre)
        self._mid = tok.encode(mid)
        self._post = tok.encode(post) + [tok.eot_id, tok.header_start] + tok.encode("assistant") + \
            [tok.header_end] + tok.encode("\n\n")

    def retrieve(self, questions: Sequence[str]):
        if self.stream is None:
            q = self.embedder.embed(questions, input_type="query")
            scores, ids = self.index.search(q, self.top_k)
            return scores.cpu(), ids.cpu()
        with torch.cuda.stream(self.stream):
            q = self.embedder.embed(questions, input_type="query")
            scores, ids = self.index.search(q, self.top_k)
            return scores.cpu(), ids.cpu()

    def context_ids(self, doc_ids: Sequence[int], scores: Sequence[float]) -> tuple:
        out: List[int] = []
        used: List[int] = []
        total = 0
        for d, s in zip(doc_ids, scores):
            if d < 0:
                continue
            if self.score_threshold is not None and s < self.score_threshold:
                continue
            ids = self.docs.token_ids(int(d), self.llm.tok)
            total += len(ids)
            if total > self.max_ctx:
                break
            if out:
                out += self.docs.sep_ids(self.llm.tok)
            out += ids
            used.append(int(d))
        return out, used

    def build_prompt(self, question: str, doc_ids, scores) -> tuple:
        ctx, used = self.context_ids(doc_ids, scores)
        return self._pre + ctx + self._mid + self.llm.tok.encode(" " + question) + self._post, used

    def submit(self, questions: Sequence[str], params: SamplingParams) -> List[RAGResult]:
        t0 = time.perf_counter()
        scores, ids = self.retrieve(questions)
        t1 = time.perf_counter()
        results = []
        for i, qtext in enumerate(questions):
            prompt, used = self.build_prompt(qtext, ids[i].tolist(), scores[i].tolist())
            req = self.llm.add_request(prompt, params)
            results.append(RAGResult(qtext, req, used, scores[i].tolist(), t0, t1, len(prompt)))
        return results

    # ------------------------------------------------------------------ non-blocking path
    def submit_async(self, questions: Sequence[str], params: SamplingParams) -> "PendingRetrieval":
        """Launch query embedding + index search on the retrieval stream and return at once;
        the top-k ids land in pinned host memory. ``poll`` turns finished retrievals into
        LLM requests. A serving loop calls ``llm.step()`` (which launches the next GPU step)
        and then ``poll()``/``submit_async()``, so neither the retrieval kernels nor the host
        work of building prompts ever leaves the GPU idle."""
        t0 = time.perf_counter()
        if self.stream is None:
            scores, ids = self.retrieve(questions)
            return PendingRetrieval(list(questions), params, scores, ids, None, t0)
        with torch.cuda.stream(self.stream):
            seqs = self.embedder.tokenize(questions, "query")
            t1 = time.perf_counter()
            q = self.embedder.embed_ids(seqs)
            t2 = time.perf_counter()
            scores, ids = self.index.search(q, self.top_k)
            t3 = time.perf_counter()
            hs = torch.empty(scores.shape, dtype=scores.dtype, pin_memory=True)
            hi = torch.empty(ids.shape, dtype=ids.dtype, pin_memory=True)
            hs.copy_(scores, non_blocking=True)
            hi.copy_(ids, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        st = self.submit_host_s
        st["tokenize"] += t1 - t0
        st["embed"] += t2 - t1
        st["search"] += t3 - t2
        st["copy"] += time.perf_counter() - t3
        return PendingRetrieval(list(questions), params, hs, hi, ev, t0, keep=(scores, ids))

    def poll(self, pending: List["PendingRetrieval"], block: bool = False) -> List[RAGResult]:
        """Turn every finished retrieval of ``pending`` into LLM requests (removed from the
        list); with ``block`` wait for all of them."""
        out: List[RAGResult] = []
        still = []
        for pr in pending:
            if pr.event is not None and not block and not pr.event.query():
                still.append(pr)
                continue
            if pr.event is not None:
                pr.event.synchronize()
            t1 = time.perf_counter()
            sc, ix = pr.scores.tolist(), pr.ids.tolist()
            for i, qtext in enumerate(pr.questions):
                prompt, used = self.build_prompt(qtext, ix[i], sc[i])
                req = self.llm.add_request(prompt, pr.params)
                t0 = pr.t0[i] if isinstance(pr.t0, list) else pr.t0
                out.append(RAGResult(qtext, req, used, sc[i], t0, t1, len(prompt)))
        pending[:] = still
        return out

    def run(self, questions: Sequence[str], params: SamplingParams) -> List[RAGResult]:
        res = self.submit(questions, params)
        self.llm.run_until_done([r.request for r in res])
        return res
