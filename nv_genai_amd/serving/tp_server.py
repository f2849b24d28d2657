"""Model-parallel model server (Llama-3-70B on 8 x MI355X; SURVEY.md §2.E "TP"/"PP", §7.2 step 7).

Launched with one process per GPU::

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m nv_genai_amd.serving.tp_server \
        --llm llama3-70b --tp 8 --port 8000

Every rank builds its weight shard (column-parallel QKV / gate-up, row-parallel O / down,
vocab-parallel embedding + LM head) and its KV-cache shard (1 of 8 kv heads per GPU). Rank 0
of each TP group runs the HTTP front end and the scheduler and broadcasts each step's layout;
the other ranks execute the same forward in :meth:`LLMEngine.run_follower`, and the
row-parallel all-reduces / vocab all-gather run over RCCL on xGMI. With ``world > tp`` the
TP groups are data-parallel replicas, each serving on ``port + replica``.

Recovery: run under ``torchrun --max-restarts N``. A rank that dies (or a driver step stuck
past ``--watchdog-s``, which the driver turns into an exit) makes the elastic agent stop the
group and start it again — fresh RCCL communicators, KV caches and weights — and the server
comes back on the same port; ``NGA_FAULT`` (utils/faults.py) injects such failures.

``--pp`` splits the layers into pipeline stages (each stage optionally TP inside): stage 0
holds the embedding + LM head and drives, activations flow stage to stage over RCCL p2p —
for models that do not fit one TP group's HBM, e.g. ``--tp 4 --pp 2``.
"""
from __future__ import annotations

import argparse
import logging
import os


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--llm", default="llama3-70b")
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--pp", type=int, default=1, help="pipeline stages (layer split)")
    ap.add_argument("--sequence-parallel", action="store_true", help="SP for long TP prefills")
    ap.add_argument("--embed", default="", help="encoder preset served by rank 0 of each replica")
    ap.add_argument("--weights", default="")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--max-num-seqs", type=int, default=128)
    ap.add_argument("--max-model-len", type=int, default=8192)
    ap.add_argument("--kv-cache-fraction", type=float, default=0.5)
    ap.add_argument("--watchdog-s", type=float, default=120.0,
                    help="a step stuck this long exits the driver so torchrun restarts the group")
    args = ap.parse_args(argv)
    logging.basicConfig(level=os.environ.get("LOGLEVEL", "INFO").upper())

    from ..engine.llm_engine import EngineConfig, LLMEngine
    from ..parallel import dist as pd

    pctx = pd.init_distributed(tp_size=args.tp, pp_size=args.pp)
    weights = None
    if args.weights:
        from ..utils.checkpoint import load_weights

        weights = load_weights(args.weights)
    eng = LLMEngine(EngineConfig(model=args.llm, max_num_seqs=args.max_num_seqs, max_model_len=args.max_model_len,
                                 kv_cache_fraction=args.kv_cache_fraction,
                                 sequence_parallel=args.sequence_parallel), pctx=pctx, weights=weights)
    if not eng.is_driver:
        eng.run_follower()
        pd.destroy()
        return
    import uvicorn

    from .engine_service import EngineService
    from .model_server import create_app

    emb = None
    if args.embed:
        from ..engine.embed_engine import EmbeddingEngine

        emb = EmbeddingEngine(args.embed)
    # fail fast: a stuck collective (dead / wedged peer) ends the process, and torchrun's
    # elastic agent (--max-restarts) restarts the whole group with fresh communicators
    svc = EngineService(eng, watchdog_s=args.watchdog_s, fail_fast=pctx.mp_size > 1)
    app = create_app(svc, emb, llm_name=f"meta/{args.llm}-instruct")
    try:
        uvicorn.run(app, host=args.host, port=args.port + pctx.dp_rank)
    finally:
        svc.shutdown()
        eng.stop_followers()
        pd.destroy()


if __name__ == "__main__":
    main()
