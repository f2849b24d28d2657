"""Five-minute RAG without a GPU (examples/5_mins_rag_no_gpu/main.py).

A single-process assistant ("Envie"): documents from a folder are split with a 2000/200
character splitter, embedded (passage model for documents, query model for questions) and
kept in a CPU flat index saved to disk — re-used on the next run with ``--use-existing``
(the reference pickles a FAISS store; here the snapshot is safetensors + JSONL, nothing is
unpickled). Answers stream from a chat model: a remote OpenAI/NIM endpoint (``--server``),
the hash embedder + fake LLM (``--offline``), or the in-process engines (``--local``).

    python -m nv_genai_amd.examples.five_min_rag.main --docs ./uploaded_docs --server http://host:8000
"""
from __future__ import annotations

import argparse
import os
import sys

from ...index.vectorstore import VectorStore
from ...rag.loaders import load_file
from ...rag.splitters import CharacterTextSplitter

SYSTEM = ("You are a helpful AI assistant named Envie. You will reply to questions only based on the context that "
          "you are provided. If something is out of context, you will refrain from replying and politely decline "
          "to respond to the user.")


def build_clients(args):
    if args.offline:
        from ...connectors.fake import FakeChatModel, HashEmbeddings

        return FakeChatModel(words=30), HashEmbeddings(256)
    if args.local:
        from ...connectors.local import LocalChatModel, LocalEmbeddings
        from ...engine.embed_engine import EmbeddingEngine
        from ...engine.llm_engine import EngineConfig, LLMEngine
        from ...serving.engine_service import EngineService

        svc = EngineService(LLMEngine(EngineConfig(model=args.llm_preset)))
        return LocalChatModel(svc), LocalEmbeddings(EmbeddingEngine(args.embed_preset))
    from ...connectors.http import ChatClient, EmbeddingsClient

    return (ChatClient(args.server, args.llm_model), EmbeddingsClient(args.server, args.embed_model))


def build_store(args, emb) -> VectorStore:
    dim = getattr(emb, "dim", None) or len(emb.embed_query("probe"))
    path = os.path.join(args.store, "vectorstore")
    if args.use_existing and os.path.exists(os.path.join(path, "index.json")):
        return VectorStore(emb, dim, "flat", "cosine", "cpu", persist_dir=path)
    vs = VectorStore(emb, dim, "flat", "cosine", "cpu")
    docs = []
    for f in sorted(os.listdir(args.docs)):
        try:
            docs += load_file(os.path.join(args.docs, f))
        except ValueError:
            continue
    chunks = CharacterTextSplitter(2000, 200).split_documents(docs)
    vs.add_documents(chunks)
    vs.save(path)
    return vs


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", default="uploaded_docs")
    ap.add_argument("--store", default=".")
    ap.add_argument("--use-existing", action="store_true")
    ap.add_argument("--server", default="https://integrate.api.nvidia.com/v1")
    ap.add_argument("--llm-model", default="meta/llama3-70b-instruct")
    ap.add_argument("--embed-model", default="nvidia/nv-embedqa-e5-v5")
    ap.add_argument("--offline", action="store_true")
    ap.add_argument("--local", action="store_true")
    ap.add_argument("--llm-preset", default="llama3-8b")
    ap.add_argument("--embed-preset", default="arctic-embed-l")
    ap.add_argument("--question", default=None, help="answer one question and exit")
    args = ap.parse_args(argv)
    llm, emb = build_clients(args)
    vs = build_store(args, emb)

    def answer(q: str):
        docs = vs.similarity_search(q, 4)
        context = "\n\n".join(d.page_content for d in docs)
        user = f"Context: {context}\n\nQuestion: {q}\n"
        for chunk in llm.stream([("system", SYSTEM), ("user", user)]):
            sys.stdout.write(chunk)
            sys.stdout.flush()
        sys.stdout.write("\n")

    if args.question:
        answer(args.question)
        return
    while True:
        try:
            q = input("> ")
        except EOFError:
            break
        if q.strip():
            answer(q)


if __name__ == "__main__":
    main()
