"""Tutorial 03 — LlamaIndex-style RAG (reference notebooks 03_Option(1)/(2)): a query engine
over an index with a node post-processor; here dense + BM25 hybrid retrieval fused with RRF
and reranked by the cross-encoder, then the 1500-token context cap of
``LimitRetrievedNodesLength`` before generation.

    python notebooks/03_hybrid_rerank_rag.py --tiny
"""
import argparse

from _stack import local_stack

from nv_genai_amd.chain_server.utils import LimitRetrievedNodesLength
from nv_genai_amd.index.vectorstore import VectorStore
from nv_genai_amd.rag.hybrid import HybridRetriever

DOCS = ["The H100 GPU has 80 GB of HBM3 memory.", "The MI355X accelerator has 288 GB of HBM3E memory.",
        "Llamas are camelids from South America.", "The Grace CPU has 72 Arm Neoverse V2 cores.",
        "RCCL implements collectives over xGMI links."]


def main(tiny=True):
    llm, emb, rr, svc, engine = local_stack(tiny)
    try:
        store = VectorStore(emb, engine.dim, device=str(engine.device))
        store.add_texts(DOCS, [{"source": f"doc{i}"} for i in range(len(DOCS))])
        hybrid = HybridRetriever(store, reranker=rr, sparse_k=10, dense_k=10, ranker_k=5)
        q = "How much memory does the MI355X have?"
        hits = hybrid.search(q, k=3, pipeline="ranked_hybrid")
        nodes = LimitRetrievedNodesLength().postprocess([d for d, _ in hits])
        ctx = "\n".join(n.page_content for n in nodes)
        answer = "".join(llm.stream([("user", f"Context: {ctx}\nQuestion: {q}")]))
        print("top passage:", hits[0][0].page_content if hits else None)
        return hits, answer
    finally:
        svc.shutdown()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiny", action="store_true")
    main(ap.parse_args().tiny)
