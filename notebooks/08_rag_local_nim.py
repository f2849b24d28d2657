"""Tutorial 08 — RAG against a locally served model (reference notebook 08: LangChain with a
local NIM endpoint): start this framework's OpenAI/NIM-compatible model server, talk to it
with the HTTP connectors (chat, embeddings, ranking) exactly as with a remote NIM.

    python notebooks/08_rag_local_nim.py --tiny
    python notebooks/08_rag_local_nim.py --url http://localhost:8000
"""
import argparse
import socket
import threading
import time

from _stack import local_stack

from nv_genai_amd.connectors.http import ChatClient, EmbeddingsClient, RerankClient
from nv_genai_amd.index.vectorstore import VectorStore


def serve(tiny):
    import uvicorn

    from nv_genai_amd.serving.model_server import create_app

    from nv_genai_amd.engine.embed_engine import EmbeddingEngine

    _, _, _, svc, emb = local_stack(tiny)
    rr = EmbeddingEngine("reranker-tiny" if tiny else "bge-reranker-large", device=str(emb.device))
    app = create_app(svc, emb, rr, llm_name="local-llm", embed_name="local-embed", rerank_name="local-rerank")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    srv = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="error"))
    threading.Thread(target=srv.run, daemon=True).start()
    while not srv.started:
        time.sleep(0.05)
    return f"http://127.0.0.1:{port}", srv, svc


def main(tiny=True, url=None):
    srv = svc = None
    if url is None:
        url, srv, svc = serve(tiny)
    try:
        chat = ChatClient(url, "local-llm", max_tokens=32)
        emb = EmbeddingsClient(url, "local-embed")
        store = VectorStore(emb, len(emb.embed_query("probe")), device="cpu")
        store.add_texts(["NIM serves models behind an OpenAI-compatible API.", "Llamas live in the Andes."])
        q = "What API does NIM expose?"
        docs = store.similarity_search(q, 2)
        ranked = RerankClient(url, "local-rerank").rank(q, [d.page_content for d in docs])
        ctx = docs[ranked[0]["index"]].page_content
        answer = chat.invoke([("user", f"Context: {ctx}\nQuestion: {q}")])
        print("context:", ctx, "| answer:", answer[:60])
        return answer
    finally:
        if srv is not None:
            srv.should_exit = True
            svc.shutdown()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiny", action="store_true")
    ap.add_argument("--url")
    a = ap.parse_args()
    main(a.tiny, a.url)
