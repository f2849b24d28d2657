"""Shared setup for the tutorials: in-process engines (the local NIM / embedding / reranking
roles). ``tiny=True`` builds random-init tiny models on the CPU so every tutorial runs in
seconds anywhere; otherwise Llama-3-8B + arctic-embed-l (+ reranker) on the GPU."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from nv_genai_amd.connectors.local import LocalChatModel, LocalEmbeddings, LocalReranker  # noqa: E402
from nv_genai_amd.engine.embed_engine import EmbeddingEngine  # noqa: E402
from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine  # noqa: E402
from nv_genai_amd.serving.engine_service import EngineService  # noqa: E402


def local_stack(tiny: bool = True, max_tokens: int = 64):
    if tiny:
        llm = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=8, max_batched_tokens=2048, max_model_len=2048,
                                     kv_cache_blocks=256), device="cpu")
        emb = EmbeddingEngine("encoder-tiny", device="cpu")
        rr = EmbeddingEngine("reranker-tiny", device="cpu")
    else:
        llm = LLMEngine(EngineConfig(model="llama3-8b"))
        emb = EmbeddingEngine("arctic-embed-l")
        rr = EmbeddingEngine("bge-reranker-large")
    svc = EngineService(llm)
    return (LocalChatModel(svc, max_tokens=max_tokens), LocalEmbeddings(emb), LocalReranker(rr, "reranker", 4),
            svc, emb)
