"""FM-radio streaming-ASR RAG chain server (SURVEY.md §2.A E2, §2.G "alternate chain-server
API"; reference: experimental/fm-asr-streaming-rag/chain-server/{server,accumulator,
database,chains,common,utils,prompts}.py).

API (same routes and payloads as the reference):
* ``POST /storeStreamingText`` {"transcript", "source_id", "timestamp"} → the text is appended
  to that source's accumulator and re-split (recursive character splitter, DB_CHUNK_SIZE 256 /
  DB_CHUNK_OVERLAP 32); every *complete* chunk (all but the last) is written to the timestamp
  DB and the vector store → {"status": "Added N entries"};
* ``GET /generate`` with a JSON body (``LLMConfig``) → streams raw text. With
  ``use_knowledge_base`` the question's intent is classified by the LLM (pydantic
  ``UserIntent``, JSON repair on failure): ``RecentSummary`` → entries of the last N time
  units (``TimeResponse``), ``TimeWindow`` → entries within ±90 s of N units ago, otherwise /
  on any failure → similarity retrieval. More than ``max_docs`` entries are reduced by
  recursive LLM summarisation (≤ 3 rounds) when ``allow_summary``, else truncated;
* ``GET /serverStatus`` → {"is_ready": true}; ``GET /availableNvidiaModels`` → the chat
  models the connected LLM exposes.

Two reference defects are fixed rather than replicated (both silently forced every time
question down the similarity path): ``TimestampDatabase.past`` used ``datetime.timedelta``
on the ``datetime`` class, and ``sanitize_time_unit`` read a global before assignment.
Unknown time units are mapped to the closest valid one by embedding similarity.
"""
from __future__ import annotations

import datetime as dt
import json
import os
import re
import sqlite3
import threading
from typing import Iterator, List, Literal, Optional

from fastapi import Request
from pydantic import BaseModel, Field

from ..index.vectorstore import Document
from ..rag.splitters import RecursiveCharacterTextSplitter

RAG_PROMPT = ("You are a query answering system specialized in providing accurate responses to questions based "
              "on a live radio transcript. Your input includes:\n- 'Transcript': a radio transcript that you're "
              "currently listening to.\n- 'User': the user query that you're responding to.\nYour task is to "
              "answer the user query by directly referencing and extracting information from these transcripts. "
              "Ensure your responses are concise and accurate.")
SUMMARIZATION_PROMPT = ("You are a sophisticated summarization tool designed to condense large blocks of text into "
                        "a concise summary. Given the user text, reduce the character count by distilling into "
                        "only the most important information.")
MAX_SUMMARIZATION_ATTEMPTS = 3
VALID_TIME_UNITS = ["seconds", "minutes", "hours", "days"]


class TextEntry(BaseModel):
    transcript: str = Field("Streaming text to store")
    source_id: str = Field("Source of text")
    timestamp: Optional[str] = None


class LLMConfig(BaseModel):
    question: str
    context: Optional[str] = None
    name: str = "local"
    engine: str = "local"
    use_knowledge_base: bool = True
    allow_summary: bool = False
    temperature: float = 0.2
    max_docs: int = 5
    num_tokens: int = 256


class TimeResponse(BaseModel):
    timeNum: float = Field(description="The number of time units the user asked about")
    timeUnit: str = Field(description="The unit of time the user asked about")


class UserIntent(BaseModel):
    intentType: Literal["SpecificTopic", "RecentSummary", "TimeWindow", "Unknown"] = Field(
        description="The intent of user's query")


def _schema(model) -> str:
    return json.dumps(model.model_json_schema())


INTENT_PROMPT = ("You are an advanced classification system designed to understand and categorize user intent "
                 "from natural language input. Your sole output is JSON, representing the classification of the "
                 "intent according to the following specification:\n\n" + _schema(UserIntent) +
                 "\n\nSpecificTopic: a question about a particular topic. RecentSummary: a request to summarize "
                 "what was said recently. TimeWindow: a question about a specific time in the past.")
RECENCY_PROMPT = ("You are an expert at restructuring natural language input into JSON. Your input is natural "
                  "language from a user and your output is JSON and nothing else. Respond in JSON per the "
                  "following specification:\n\n" + _schema(TimeResponse))


def sanitize_json(text: str, model=None) -> Optional[str]:
    """Replace quote/escape mistakes, then return the first substring that parses as JSON
    (and validates against ``model`` when given)."""
    t = text.replace("'", '"').replace("\\_", "_")
    for m in re.findall(r"(\{.*?\}|\[.*?\])", t, re.DOTALL):
        try:
            json.loads(m)
            if model is not None:
                model.model_validate_json(m)
            return m
        except (json.JSONDecodeError, ValueError):
            continue
    return None


def classify(question: str, llm, system: str, model):
    out = llm.invoke([("system", system), ("user", question)])
    try:
        return model.model_validate_json(out)
    except ValueError:
        fixed = sanitize_json(out, model)
        if fixed is None:
            return None
        try:
            return model.model_validate_json(fixed)
        except ValueError:
            return None


class TimestampDatabase:
    """Time-indexed transcript chunks (SQLite, thread-safe)."""

    def __init__(self, path: str = ":memory:"):
        self.conn = sqlite3.connect(path, check_same_thread=False)
        self.lock = threading.Lock()
        with self.lock:
            self.conn.execute("CREATE TABLE IF NOT EXISTS messages (id INTEGER PRIMARY KEY, text TEXT, "
                              "timestamp TEXT, source_id TEXT)")
            self.conn.execute("CREATE INDEX IF NOT EXISTS ts ON messages(timestamp)")
            self.conn.commit()

    @staticmethod
    def _fmt(t: dt.datetime) -> str:
        return t.strftime("%Y-%m-%d %H:%M:%S.%f")

    def insert_docs(self, docs: List[str], source_id: str, tnow: Optional[dt.datetime] = None):
        tnow = tnow or dt.datetime.now()
        with self.lock:
            self.conn.executemany("INSERT INTO messages (text, timestamp, source_id) VALUES (?, ?, ?)",
                                  [(d, self._fmt(tnow), source_id) for d in docs])
            self.conn.commit()

    def _rows(self, sql: str, args) -> List[Document]:
        with self.lock:
            rows = self.conn.execute(sql, args).fetchall()
        return [Document(r[1], {"tstamp": dt.datetime.strptime(r[2], "%Y-%m-%d %H:%M:%S.%f"), "source_id": r[3]})
                for r in rows]

    def recent(self, tstamp: dt.datetime) -> List[Document]:
        return self._rows("SELECT * FROM messages WHERE timestamp >= ? ORDER BY timestamp", (self._fmt(tstamp),))

    def past(self, tstamp: dt.datetime, window: float = 90) -> List[Document]:
        a, b = tstamp - dt.timedelta(seconds=window), tstamp + dt.timedelta(seconds=window)
        return self._rows("SELECT * FROM messages WHERE timestamp BETWEEN ? AND ? ORDER BY timestamp",
                          (self._fmt(a), self._fmt(b)))


class TextAccumulator:
    def __init__(self, store, chunk_size: int = 256, chunk_overlap: int = 32, db: Optional[TimestampDatabase] = None):
        self.splitter = RecursiveCharacterTextSplitter(chunk_size, chunk_overlap)
        self.acc: dict = {}
        self.db = db or TimestampDatabase()
        self.store = store
        self.lock = threading.Lock()

    def update(self, source_id: str, text: str) -> dict:
        with self.lock:
            docs = self.splitter.split_text(f"{self.acc.get(source_id, '')} {text}")
            if not docs:
                return {"status": "Added 0 entries"}
            self.acc[source_id], new = docs[-1], docs[:-1]
            if new:
                self.db.insert_docs(new, source_id)
                self.store.add_texts(new, [{"source_id": source_id, "source": source_id}] * len(new))
        return {"status": f"Added {len(new)} entries"}


class RagChain:
    def __init__(self, cfg: LLMConfig, acc: TextAccumulator, llm, embedder=None):
        self.cfg, self.acc, self.llm, self.embedder = cfg, acc, llm, embedder
        self.db = acc.db

    def _stream(self, system: Optional[str], user: str) -> Iterator[str]:
        msgs = ([("system", system)] if system else []) + [("user", user)]
        yield from self.llm.stream(msgs, temperature=self.cfg.temperature, max_tokens=self.cfg.num_tokens)

    def generate(self, docs: List[Document]) -> Iterator[str]:
        ctx = "\n".join(d.page_content for d in docs)
        yield from self._stream(RAG_PROMPT, f"Transcript: '{ctx}'\nUser: '{self.cfg.question}'\nAI:")

    def time_unit(self, unit: str) -> str:
        u = unit.lower().strip()
        if u in VALID_TIME_UNITS:
            return u
        if u + "s" in VALID_TIME_UNITS:
            return u + "s"
        if self.embedder is not None:
            import torch

            v = self.embedder.embed_documents(VALID_TIME_UNITS + [u])
            t = torch.tensor(v)
            t = t / t.norm(dim=1, keepdim=True)
            return VALID_TIME_UNITS[int((t[:-1] @ t[-1]).argmax())]
        for v in VALID_TIME_UNITS:
            if v.startswith(u[:3]):
                return v
        raise ValueError(f"unknown time unit {unit!r}")

    def seconds(self, r: TimeResponse) -> float:
        return dt.timedelta(**{self.time_unit(r.timeUnit): r.timeNum}).total_seconds()

    def answer(self) -> Iterator[str]:
        if not self.cfg.use_knowledge_base:
            yield from self._stream(None, self.cfg.question)
            return
        intent = classify(self.cfg.question, self.llm, INTENT_PROMPT, UserIntent)
        if intent is not None and intent.intentType in ("RecentSummary", "TimeWindow"):
            try:
                rec = classify(self.cfg.question, self.llm, RECENCY_PROMPT, TimeResponse)
                if rec is None:
                    raise ValueError("could not parse the time range")
                if intent.intentType == "RecentSummary":
                    yield from self.answer_by_recent(rec)
                else:
                    yield from self.answer_by_past(rec)
                return
            except Exception:  # noqa: BLE001 - fall back to similarity retrieval like the reference
                pass
        yield from self.answer_by_relevance()

    def answer_by_relevance(self) -> Iterator[str]:
        docs = self.acc.store.similarity_search(self.cfg.question, self.cfg.max_docs) if len(self.acc.store) else []
        if not docs:
            yield "*Found no documents related to the query*"
            return
        yield f"*Returned {len(docs)} related entries*\n\n"
        yield from self.generate(docs)

    def _reduce(self, docs: List[Document]) -> Iterator:
        """Yield progress lines; the reduced docs are returned through StopIteration.value."""
        if len(docs) <= self.cfg.max_docs:
            return docs
        if self.cfg.allow_summary:
            yield "*Using summarization to reduce context*\n"
            for attempt in range(MAX_SUMMARIZATION_ATTEMPTS):
                docs = self.summarize(docs)
                yield f"*Reduced to {len(docs)} entries on attempt {attempt + 1}*\n"
                if len(docs) <= self.cfg.max_docs:
                    break
            return docs[-self.cfg.max_docs:]
        docs = docs[-self.cfg.max_docs:]
        yield f"*Reduced to last {len(docs)} entries*\n"
        return docs

    def answer_by_recent(self, rec: TimeResponse) -> Iterator[str]:
        s = self.seconds(rec)
        docs = self.db.recent(dt.datetime.now() - dt.timedelta(seconds=s))
        yield f"*Found {len(docs)} entries from the last {s:.0f}s*\n"
        docs = yield from self._reduce(docs)
        if docs:
            yield "\n"
            yield from self.generate(docs)

    def answer_by_past(self, rec: TimeResponse, window: float = 90) -> Iterator[str]:
        s = self.seconds(rec)
        t = dt.datetime.now() - dt.timedelta(seconds=s)
        docs = self.db.past(t, window)
        yield f"*Found {len(docs)} entries from {s:.0f}s ago (+/- {window:.0f}s)*\n"
        if len(docs) > self.cfg.max_docs and not self.cfg.allow_summary:
            docs = sorted(docs, key=lambda d: abs(d.metadata["tstamp"] - t))[: self.cfg.max_docs]
            yield f"*Reduced to {len(docs)} entries closest to that time*\n"
        else:
            docs = yield from self._reduce(docs)
        if docs:
            yield "\n"
            yield from self.generate(docs)

    def summarize(self, docs: List[Document]) -> List[Document]:
        summary = ""
        for i in range(0, len(docs), self.cfg.max_docs):
            text = " ".join(d.page_content for d in docs[i:i + self.cfg.max_docs])
            summary = f"{summary} {self.llm.invoke([('system', SUMMARIZATION_PROMPT), ('user', text)])}"
        sp = RecursiveCharacterTextSplitter(self.acc.splitter.chunk_size, 0)
        return [Document(c) for c in sp.split_text(summary)]


def create_app(llm, store, embedder=None, chunk_size: Optional[int] = None, chunk_overlap: Optional[int] = None,
               db_path: str = ":memory:"):
    from fastapi import FastAPI
    from fastapi.responses import JSONResponse, StreamingResponse

    acc = TextAccumulator(store, int(chunk_size or os.environ.get("DB_CHUNK_SIZE", 256)),
                          int(chunk_overlap or os.environ.get("DB_CHUNK_OVERLAP", 32)), TimestampDatabase(db_path))
    app = FastAPI(title="FM-ASR streaming RAG chain server")
    app.state.accumulator = acc

    @app.get("/availableNvidiaModels")
    def models():
        names = getattr(llm, "available_models", None)
        return JSONResponse({"models": list(names() if callable(names) else [getattr(llm, "model", "local")])})

    @app.get("/serverStatus")
    def status():
        return {"is_ready": True}

    @app.post("/storeStreamingText")
    def store_text(data: TextEntry):
        return JSONResponse(acc.update(data.source_id, data.transcript))

    @app.get("/generate")
    async def generate(request: Request):
        cfg = LLMConfig(**json.loads(await request.body()))
        return StreamingResponse(RagChain(cfg, acc, llm, embedder).answer(), media_type="text/plain")

    return app
