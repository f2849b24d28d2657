"""Tutorial 05 — RAG over HTML documentation (reference notebook 05: fetch HTML pages,
strip markup, split, embed into FAISS, answer with a chat model). Pages come from local
files or URLs; markup is removed by the loader's HTML text extractor.

    python notebooks/05_html_rag.py --tiny
    python notebooks/05_html_rag.py --urls https://docs.example.org/a.html,...
"""
import argparse

from _stack import local_stack

from nv_genai_amd.index.vectorstore import VectorStore
from nv_genai_amd.ingest.streaming import HTTPCache
from nv_genai_amd.rag.loaders import html_to_text
from nv_genai_amd.rag.splitters import RecursiveCharacterTextSplitter

PAGE = ("<html><head><title>Triton</title><script>var x=1;</script></head><body><h1>Triton Inference Server</h1>"
        "<p>Triton supports dynamic batching with a max queue delay.</p><p>Models are loaded from a model "
        "repository.</p></body></html>")


def main(tiny=True, urls=None):
    llm, emb, _, svc, engine = local_stack(tiny)
    try:
        pages = [HTTPCache(None).get(u, 10.0) for u in urls] if urls else [PAGE]
        texts = [html_to_text(p) for p in pages]
        store = VectorStore(emb, engine.dim, device=str(engine.device))
        sp = RecursiveCharacterTextSplitter(1000, 0)
        for i, t in enumerate(texts):
            store.add_texts(sp.split_text(t), [{"source": (urls or ["inline"])[i]}] * len(sp.split_text(t)))
        q = "Does Triton support dynamic batching?"
        ctx = "\n".join(d.page_content for d in store.similarity_search(q, 4))
        answer = "".join(llm.stream([("system", "Answer using the documentation."), ("user", f"{ctx}\n\n{q}")]))
        print("context starts:", ctx[:60], "| answer:", answer[:60])
        return texts
    finally:
        svc.shutdown()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiny", action="store_true")
    ap.add_argument("--urls")
    a = ap.parse_args()
    main(a.tiny, a.urls.split(",") if a.urls else None)
