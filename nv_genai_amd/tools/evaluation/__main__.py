"""``python -m nv_genai_amd.tools.evaluation`` (tools/evaluation/rag_evaluator/main.py,
synthetic_data_generator/main.py): generate synthetic QA, generate answers through a chain
server, evaluate with RAGAS-style metrics or an LLM judge.

The LLM / embedder used for generation and judging are the framework's HTTP clients pointed
at a model server (``--model_server``), or the in-process engines (``--local``)."""
from __future__ import annotations

import argparse
import logging


def _clients(args):
    if args.local:
        from ...connectors.local import LocalChatModel, LocalEmbeddings
        from ...engine.embed_engine import EmbeddingEngine
        from ...engine.llm_engine import EngineConfig, LLMEngine
        from ...serving.engine_service import EngineService

        svc = EngineService(LLMEngine(EngineConfig(model=args.llm_preset)))
        return LocalChatModel(svc, temperature=0.1, max_tokens=300), LocalEmbeddings(EmbeddingEngine(args.embed_preset))
    from ...connectors.http import ChatClient, EmbeddingsClient

    return (ChatClient(args.model_server, args.llm_model, temperature=0.1, top_p=1.0, max_tokens=300),
            EmbeddingsClient(args.model_server, args.embed_model))


def main(argv=None):
    ap = argparse.ArgumentParser(prog="nv_genai_amd.tools.evaluation")
    ap.add_argument("--base_url", default="localhost:8081", help="chain server host:port")
    ap.add_argument("--model_server", default="http://localhost:8000", help="OpenAI-compatible model server")
    ap.add_argument("--local", action="store_true", help="use in-process engines instead of --model_server")
    ap.add_argument("--llm_model", default="meta/llama3-8b-instruct")
    ap.add_argument("--embed_model", default="snowflake/arctic-embed-l")
    ap.add_argument("--llm_preset", default="llama3-8b")
    ap.add_argument("--embed_preset", default="arctic-embed-l")
    ap.add_argument("--generate_data", action="store_true")
    ap.add_argument("--generate_answer", action="store_true")
    ap.add_argument("--evaluate", action="store_true")
    ap.add_argument("--metrics", default="ragas", choices=["ragas", "judge_llm"])
    ap.add_argument("--docs", default="", help="dataset folder")
    ap.add_argument("--gt", default="qna.json", help="synthetic QA file")
    ap.add_argument("--ev", default="eval.json", help="evaluation file (answers)")
    ap.add_argument("--result", default="result", help="result path prefix")
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    llm, emb = _clients(args)
    if args.generate_data:
        from .data_generator import generate_synthetic_data

        generate_synthetic_data(args.docs, args.gt, llm)
    if args.generate_answer:
        from .answer_generator import generate_answers

        generate_answers(args.base_url, args.docs, args.gt, args.ev)
    if args.evaluate:
        from .evaluator import eval_llm_judge, eval_ragas

        res = eval_ragas(args.ev, args.result, emb, llm) if args.metrics == "ragas" else eval_llm_judge(args.ev, args.result, llm)
        print(res)


if __name__ == "__main__":
    main()
