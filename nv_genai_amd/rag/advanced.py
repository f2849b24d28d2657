"""Advanced retrieval strategies.

ORAN / multimodal-assistant chatbots (experimental/oran-chatbot-multimodal/
Multimodal_Assistant.py:92-160,395-590; retriever/retriever.py:85-148;
guardrails/fact_check.py:28-38; utils/memory.py:19-47; utils/feedback.py:28-46):

* ``rag_type`` 0 — plain score-threshold retrieval (k 10, threshold 0.3);
* 1 — **multi-query**: the LLM writes alternative phrasings, every query is searched,
  duplicates are dropped (first source kept) and a cross-encoder keeps the best 10;
* 2 — **HyDE**: the query is extended with an LLM-written hypothetical answer before search,
  then the same dedupe + rerank;
* 3 — multi-query through a line-list parser (the LangChain ``MultiQueryRetriever`` flavour);
* **query rewriting** of follow-ups against the conversation summary;
* **conversation summary memory** (rolling LLM summary of the chat);
* **fact-check guardrail** (a second LLM pass that prefixes TRUE/FALSE);
* **feedback** log (5-face score + comment; JSONL instead of a Google sheet).

RAG developer chatbot (experimental/rag-developer-chatbot/notebooks): ``MergerRetriever``
(lord-of-the-retrievers: interleave several retrievers), ``EmbeddingsRedundantFilter``
(drop near-duplicate passages, cosine ≥ 0.95) and ``EmbeddingsFilter`` contextual compression
(keep passages whose similarity to the query ≥ threshold) — all batched as one GEMM on the
embedding device instead of per-pair Python loops.
"""
from __future__ import annotations

import datetime
import json
import os
import re
import threading
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch

from ..index.vectorstore import Document

MULTI_QUERY_PROMPT = ("You are a helpful expert assistant. Your task is to generate five different versions of "
                      "the given user question to retrieve relevant documents from a vector database. By "
                      "generating multiple perspectives on the user question, your goal is to help the user "
                      "overcome some of the limitations of the distance-based similarity search. Provide these "
                      "alternative questions separated by newlines.\nOriginal question: {question}")
HYDE_PROMPT = ("You are a helpful expert assistant. Provide an example answer to the given question, that "
               "might be found in a document.")
REWRITE_PROMPT = ("Here is the conversation history between user and Assistant. User has a follow-up question "
                  "to the conversation. Your task is to rewrite user's follow-up question based on the given "
                  "conversation history. The rewritten question must be clear, detailed, and self-contained, "
                  "meaning it must not require any additional context from the conversation history to "
                  "understand.")
SUMMARY_PROMPT = ("Progressively summarize the lines of conversation provided, adding onto the previous summary "
                  "returning a new summary.\n\nCurrent summary:\n{summary}\n\nNew lines of conversation:\n"
                  "{new_lines}\n\nNew summary:")
FACT_CHECK_PROMPT = ("Your task is to conduct a thorough fact-check of a response provided by a large language "
                     "model. You will be given the context documents as [[CONTEXT]], the original question posed "
                     "by the user as [[QUESTION]], and the model's response as [[RESPONSE]]. Verify each part of "
                     "the response against the context only. If your fact check returns True, start your reply "
                     "with '**:green[TRUE]**', and if it returns False, start your reply with '**:red[FALSE]**'.")


def _invoke(llm, system: Optional[str], user: str) -> str:
    msgs = ([("system", system)] if system else []) + [("user", user)]
    return llm.invoke(msgs)


def parse_lines(text: str) -> List[str]:
    """LLM list output → clean queries (numbering/bullets stripped, preamble lines dropped)."""
    out = []
    for ln in text.strip().split("\n"):
        ln = re.sub(r"^\s*(?:\d+[.)]|[-*•])\s*", "", ln).strip().strip('"')
        if not ln or ln.endswith(":"):
            continue
        out.append(ln)
    return out


def augment_multiple_query(llm, query: str) -> List[str]:
    return parse_lines(_invoke(llm, None, MULTI_QUERY_PROMPT.format(question=query)))


def augment_query_generated(llm, query: str) -> str:
    return _invoke(llm, HYDE_PROMPT, query)


def query_rewriting(llm, query: str, history: str) -> str:
    return _invoke(llm, REWRITE_PROMPT, f"Conversation history:\n{history}\n\nFollow-up question: {query}")


def dedupe(docs: Sequence[Document]) -> List[Document]:
    seen, out = set(), []
    for d in docs:
        if d.page_content not in seen:
            seen.add(d.page_content)
            out.append(d)
    return out


def rerank_top(reranker, query: str, docs: Sequence[Document], n: int = 10) -> List[Document]:
    if reranker is None or not docs:
        return list(docs)[:n]
    ranks = reranker.rank(query, [d.page_content for d in docs])
    return [docs[r["index"]] for r in ranks[:n]]


def sources_of(docs: Sequence[Document]) -> Dict[str, dict]:
    """{source: {"doc_content", "doc_metadata"}}; passages of one source are concatenated."""
    out: Dict[str, dict] = {}
    for d in docs:
        src = d.metadata.get("source") or d.metadata.get("filename", "")
        if src in out:
            out[src]["doc_content"] += "\n\n" + d.page_content
        else:
            out[src] = {"doc_content": d.page_content, "doc_metadata": src}
    return out


class AdvancedRetriever:
    """The four ``rag_type`` strategies over one vector store (+ optional cross-encoder)."""

    def __init__(self, store, llm, reranker=None, k: int = 10, score_threshold: float = 0.3, top_n: int = 10):
        self.store, self.llm, self.reranker = store, llm, reranker
        self.k, self.threshold, self.top_n = k, score_threshold, top_n

    def _search(self, queries: Sequence[str]) -> List[Document]:
        hits = self.store.similarity_search_with_score_batch(list(queries), self.k)   # one batched search
        out = []
        for row in hits:
            out += [d for d, s in row if self.store.relevance(s) >= self.threshold]
        return out

    def retrieve(self, query: str, rag_type: int = 0) -> Tuple[List[Document], str, Dict[str, dict]]:
        if rag_type == 0:
            docs = self._search([query])
        elif rag_type in (1, 3):
            docs = rerank_top(self.reranker, query,
                              dedupe(self._search([query] + augment_multiple_query(self.llm, query))), self.top_n)
        elif rag_type == 2:
            hyde = query + " " + augment_query_generated(self.llm, query)
            docs = rerank_top(self.reranker, query, dedupe(self._search([hyde])), self.top_n)
        else:
            raise ValueError(f"unknown rag_type {rag_type}")
        context = "".join(d.page_content + "\n\n" for d in docs)
        return docs, context, sources_of(docs)


class MergerRetriever:
    """Round-robin merge of several retrievers' ranked lists (rank 0 of each, then rank 1...)."""

    def __init__(self, retrievers: Sequence):
        self.retrievers = list(retrievers)

    def invoke(self, query: str) -> List[Document]:
        lists = [r.invoke(query) for r in self.retrievers]
        out = []
        for i in range(max((len(x) for x in lists), default=0)):
            out += [x[i] for x in lists if i < len(x)]
        return out


class EmbeddingsRedundantFilter:
    def __init__(self, embedder, threshold: float = 0.95):
        self.embedder, self.threshold = embedder, threshold

    def transform_documents(self, docs: Sequence[Document]) -> List[Document]:
        if len(docs) < 2:
            return list(docs)
        e = _embed(self.embedder, [d.page_content for d in docs])
        sim = e @ e.t()
        keep = []
        for i in range(len(docs)):
            if all(float(sim[i, j]) < self.threshold for j in keep):
                keep.append(i)
        return [docs[i] for i in keep]


class EmbeddingsFilter:
    def __init__(self, embedder, similarity_threshold: float = 0.5):
        self.embedder, self.threshold = embedder, similarity_threshold

    def compress_documents(self, docs: Sequence[Document], query: str) -> List[Document]:
        if not docs:
            return []
        e = _embed(self.embedder, [d.page_content for d in docs])
        q = _embed(self.embedder, [query], query=True)
        s = (e @ q.t()).squeeze(1)
        return [d for d, v in zip(docs, s.tolist()) if v >= self.threshold]


class ContextualCompressionRetriever:
    def __init__(self, base, compressors: Sequence):
        self.base, self.compressors = base, list(compressors)

    def invoke(self, query: str) -> List[Document]:
        docs = self.base.invoke(query)
        for c in self.compressors:
            docs = c.compress_documents(docs, query) if hasattr(c, "compress_documents") else c.transform_documents(docs)
        return docs


def _embed(embedder, texts: Sequence[str], query: bool = False) -> torch.Tensor:
    if query and hasattr(embedder, "embed_query_tensor"):
        e = embedder.embed_query_tensor(list(texts))
    elif not query and hasattr(embedder, "embed_documents_tensor"):
        e = embedder.embed_documents_tensor(list(texts))
    else:
        f = embedder.embed_query if query else None
        e = torch.tensor([f(t) for t in texts] if f else embedder.embed_documents(list(texts)))
    e = e.float()
    return e / e.norm(dim=-1, keepdim=True).clamp_min(1e-12)


class SummaryMemory:
    """Rolling conversation summary (ConversationSummaryMemory)."""

    def __init__(self, llm, prompt: str = SUMMARY_PROMPT):
        self.llm, self.prompt, self.buffer = llm, prompt, ""
        self.messages: List[Tuple[str, str]] = []

    def add(self, user: str, ai: str) -> str:
        self.messages += [("user", user), ("assistant", ai)]
        lines = f"Human: {user}\nAI: {ai}"
        self.buffer = self.llm.invoke([("user", self.prompt.format(summary=self.buffer, new_lines=lines))])
        return self.buffer


def fact_check(llm, evidence: str, query: str, response: str):
    """Streams the fact-check verdict (starts with TRUE/FALSE marker)."""
    user = f"[[CONTEXT]]\n\n{evidence}\n\n[[QUESTION]]\n\n{query}\n\n[[RESPONSE]]\n\n{response}"
    return llm.stream([("system", FACT_CHECK_PROMPT), ("user", user)])


FACES = {"😀": 5, "🙂": 4, "😐": 3, "🙁": 2, "😞": 1}


class FeedbackLog:
    def __init__(self, path: str):
        self.path = path
        self._lock = threading.Lock()

    def submit(self, feedback: dict, query: str, response: str) -> dict:
        score = FACES.get(feedback.get("score"), feedback.get("score"))
        row = {"time": datetime.datetime.now().strftime("%Y-%m-%d %H:%M:%S"), "score": score, "query": query,
               "response": response, "comment": f"Score: {score}/5. Feedback: {feedback.get('text') or 'none'}"}
        with self._lock:
            os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)
            with open(self.path, "a") as f:
                f.write(json.dumps(row, ensure_ascii=False) + "\n")
        return row


class AdvancedRAGChat:
    """End-to-end ORAN-style turn: rewrite follow-up → retrieve (rag_type) → answer → update
    summary memory → optional fact check."""

    def __init__(self, retriever: AdvancedRetriever, llm, header: str, fact_checking: bool = True,
                 rewrite: bool = True):
        self.r, self.llm, self.header = retriever, llm, header
        self.memory = SummaryMemory(llm)
        self.fact_checking, self.rewrite = fact_checking, rewrite

    def ask(self, question: str, rag_type: int = 0, on_chunk: Optional[Callable[[str], None]] = None) -> dict:
        q = question
        if self.rewrite and self.memory.buffer:
            q = query_rewriting(self.llm, question, self.memory.buffer)
        docs, context, sources = self.r.retrieve(q, rag_type)
        prompt = "Relevant documents:" + context + "\n\n[[QUESTION]]\n\n" + q
        answer = ""
        for c in self.llm.stream([("system", self.header), ("user", prompt)]):
            answer += c
            if on_chunk:
                on_chunk(c)
        self.memory.add(q, answer)
        check = "".join(fact_check(self.llm, context, q, answer)) if self.fact_checking else None
        return {"query": q, "answer": answer, "sources": sources, "fact_check": check}
