"""Tutorial 02 — minimalistic RAG (reference notebooks 02_Option(1)/(2)): split a text,
embed the chunks into a vector store, retrieve the top-k for a question and answer with a
chat model — here the in-process Llama engine instead of a hosted endpoint or an HF pipeline.

    python notebooks/02_simple_rag.py --tiny
"""
import argparse

from _stack import local_stack

from nv_genai_amd.index.vectorstore import VectorStore
from nv_genai_amd.rag.splitters import RecursiveCharacterTextSplitter

TEXT = ("Sweden is a Nordic country in Northern Europe. Its capital is Stockholm. The population is about ten "
        "million. Sweden is a constitutional monarchy with a parliamentary system. ") * 8
PROMPT = ("Answer solely based on the following context:\n<Documents>\n{context}\n</Documents>\n\nQuestion: {q}")


def main(tiny=True):
    llm, emb, _, svc, engine = local_stack(tiny)
    try:
        store = VectorStore(emb, engine.dim, device=str(engine.device))
        store.add_texts(RecursiveCharacterTextSplitter(400, 50).split_text(TEXT))
        q = "What is the capital of Sweden?"
        docs = store.similarity_search(q, 4)
        answer = "".join(llm.stream([("user", PROMPT.format(context="\n".join(d.page_content for d in docs), q=q))]))
        print(f"retrieved {len(docs)} chunks; answer: {answer[:100]!r}")
        return answer
    finally:
        svc.shutdown()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiny", action="store_true")
    main(ap.parse_args().tiny)
