"""Tensor-parallel Llama on the GPU box: two TP ranks share the box's one MI355X, their
row-parallel all-reduces go through the IPC custom all-reduce (csrc/kernels/custom_ar.hip),
and step broadcasts / the vocab all-gather go over gloo (RCCL refuses two ranks on one
device). The TP=2 prefill logits must match a single-process model with the same weights,
and the TP engine must generate through the custom all-reduce without falling back."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# llama-small's TP=2 rank shapes, every projection on the decode-shape kernel: K-split q/k/v
# (RoPE sums the slabs), K-split o / down (summed before the all-reduce), SwiGLU gate/up, fp32
# vocab-shard LM head
SKINNY_TP2_TABLE = {"arch": "gfx950", "table": {
    "768x1024": {"shape": "qkv", "by_m": {"16": [3, 2], "512": [1, 2]}},
    "1024x512": {"shape": "o", "by_m": {"16": [3, 2], "512": [1, 2]}},
    "2816x1024": {"shape": "gate_up", "by_m": {"16": [2, 1], "512": [13, 1]}},
    "1024x1408": {"shape": "down", "by_m": {"16": [3, 2], "512": [1, 2]}},
    "16384x1024": {"shape": "lm_head", "by_m": {"16": [2, 1], "512": [12, 1]}}}}


def _worker(rank, port, q, table=None):
    os.environ.update(RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    if table:
        os.environ["NGA_SKINNY_TABLE"] = table
    res = {"rank": rank}
    try:
        from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine, SamplingParams
        from nv_genai_amd.models.config import llama_config
        from nv_genai_amd.models.llama import AttnMeta, LlamaModel
        from nv_genai_amd.parallel import comm
        from nv_genai_amd.parallel import dist as pd

        cfg = llama_config("llama-small")
        full = LlamaModel(cfg, "cpu", dtype=torch.bfloat16, pctx=pd.ParallelContext(), seed=5).state_dict()
        full["lm_head.weight"] = full["lm_head.weight"] * 40.0  # peaky logits (as test_engine_gpu)
        pctx = pd.init_distributed(tp_size=2, backend="gloo", device="cuda")
        car = comm.custom_all_reduce_for(pctx.tp_group)
        res["custom_ar"] = car is not None and car.enabled
        dev = torch.device("cuda", 0)
        ecfg = EngineConfig(model="llama-small", max_num_seqs=4, max_batched_tokens=1024, max_model_len=1024,
                            kv_cache_blocks=64, use_graphs=False)
        eng = LLMEngine(ecfg, device="cuda", pctx=pctx, weights=full)
        # 1) prefill logits of one 200-token prompt through the TP model (every rank runs it)
        T = 200
        ids = torch.arange(10, 10 + T, dtype=torch.int32, device=dev)
        pos = torch.arange(T, dtype=torch.int32, device=dev)
        bt = torch.arange(4, dtype=torch.int32, device=dev).view(1, 4)
        meta = AttnMeta(kind="prefill", slots=torch.arange(T, dtype=torch.int32, device=dev),
                        cu_q=torch.tensor([0, T], dtype=torch.int32, device=dev),
                        ctx_lens=torch.tensor([T], dtype=torch.int32, device=dev), block_tables=bt,
                        max_q_len=T, max_ctx=T)
        lg = eng.model.logits(eng.model.forward(ids, pos, meta)).float()
        res["skinny_picks"] = sum(eng.model._pick(eng.model.layers[0][n], T) is not None
                                  for n in ("wqkv", "wo", "wgu", "wd"))
        if rank == 0:
            single = LlamaModel(cfg, dev, pctx=pd.ParallelContext(), weights=full)
            single.allocate_kv_cache(8)
            ref = single.logits(single.forward(ids, pos, meta)).float()
            res["max_abs_diff"] = float((lg - ref).abs().max())
            res["ref_abs_max"] = float(ref.abs().max())
            res["argmax_agree"] = float((lg.argmax(-1) == ref.argmax(-1)).float().mean())
            del single
        # 2) the TP engine generates (driver + follower) through the custom all-reduce
        if eng.is_driver:
            out = eng.generate([[5, 6, 7, 8] * 30, [9, 10, 11] * 20],
                               SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True))
            eng.stop_followers()
            res["gen_lens"] = [len(r.output_ids) for r in out]
        else:
            eng.run_follower()
        torch.cuda.synchronize()
        res["ar_error"] = car.error() if car is not None else -1
        pd.destroy()
    except Exception as e:  # noqa: BLE001
        import traceback

        res["exc"] = traceback.format_exc()[-3000:]
    q.put(res)


@pytest.mark.parametrize("skinny", [False, True])
def test_tp2_on_one_gpu_with_custom_all_reduce(skinny, tmp_path):
    """``skinny``: the rank-shard projections run the decode-shape kernel (test table), K-split
    row-parallel partials summed before the custom all-reduce."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    import json

    table = None
    if skinny:
        table = str(tmp_path / "skinny_tp2.json")
        with open(table, "w") as f:
            json.dump(SKINNY_TP2_TABLE, f)
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, port, q, table)) for r in range(2)]
    for p in procs:
        p.start()
    results = sorted([q.get(timeout=200) for _ in range(2)], key=lambda r: r["rank"])
    for p in procs:
        p.join(timeout=60)
    print(results)
    for r in results:
        assert "exc" not in r, r["exc"]
        assert r["custom_ar"], r
        assert r["ar_error"] == 0, r
    r0 = results[0]
    assert r0["skinny_picks"] == (4 if skinny else 0), r0
    assert r0["gen_lens"] == [8, 8]
    assert r0["max_abs_diff"] <= 0.05 * r0["ref_abs_max"] + 0.05, r0
    assert r0["argmax_agree"] >= 0.9, r0


def _graph_worker(rank, port, q):
    """TP=2 engine with decode graphs AND prefill / mixed step graphs captured on both ranks
    (every collective in them is an IPC kernel: custom all-reduce, fused add+RMSNorm, the
    logits all-gather), pipelined steps over the shared-memory channel."""
    os.environ.update(RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    res = {"rank": rank}
    try:
        from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine, SamplingParams
        from nv_genai_amd.models.config import llama_config
        from nv_genai_amd.models.llama import LlamaModel
        from nv_genai_amd.parallel import comm
        from nv_genai_amd.parallel import dist as pd

        cfg = llama_config("llama-small")
        full = LlamaModel(cfg, "cpu", dtype=torch.bfloat16, pctx=pd.ParallelContext(), seed=5).state_dict()
        full["lm_head.weight"] = full["lm_head.weight"] * 40.0  # peaky logits: no greedy near-ties
        prompts = [[5, 6, 7, 8] * 30, [9, 10, 11] * 20, [12, 13] * 70]
        greedy = SamplingParams(temperature=0.0, max_tokens=12, ignore_eos=True)
        hot = SamplingParams(temperature=0.8, top_p=0.9, max_tokens=12, ignore_eos=True, seed=3)
        ecfg = EngineConfig(model="llama-small", max_num_seqs=4, max_batched_tokens=1024, max_model_len=1024,
                            kv_cache_blocks=64, use_graphs=True, mixed_graphs=True, graph_token_step=128,
                            mixed_prefill_tokens=512)
        if rank == 0:
            import dataclasses

            e1 = LLMEngine(dataclasses.replace(ecfg, use_graphs=False, mixed_graphs=False), device="cuda",
                           pctx=pd.ParallelContext(), weights=full)
            res["ref"] = [r.output_ids for r in e1.generate(prompts, greedy)]
            del e1
            torch.cuda.empty_cache()
        pctx = pd.init_distributed(tp_size=2, backend="gloo", device="cuda")
        car = comm.custom_all_reduce_for(pctx.tp_group)
        res["custom_ar"] = car is not None and car.enabled
        eng = LLMEngine(ecfg, device="cuda", pctx=pctx, weights=full)
        res["async"] = eng.cfg.async_decode
        res["use_graphs"] = eng.cfg.use_graphs
        res["mixed_graphs_ok"] = eng._mg_ok
        if eng.is_driver:
            res["out"] = [r.output_ids for r in eng.generate(prompts, greedy)]
            res["hot"] = [r.output_ids for r in eng.generate(prompts, hot)]
            res["unpipelined"] = eng.stats["unpipelined_steps"]
            eng.stop_followers()
        else:
            eng.run_follower()
            res["gathers"] = eng._tp_gathers
        torch.cuda.synchronize()
        res["decode_graphs"] = len(eng.graphs)
        res["step_graphs"] = len(eng.mgraphs)
        res["last_tok"] = eng.d_tok[:3].tolist()
        res["gather_calls"] = car.gather_count if car is not None else 0
        # the same TP=2 replica eager and synchronous: the same kernels in the same order, so
        # the graphed pipelined run must reproduce it token for token
        import dataclasses

        e2 = LLMEngine(dataclasses.replace(ecfg, use_graphs=False, mixed_graphs=False, async_decode=False),
                       device="cuda", pctx=pctx, model=eng.model, tokenizer=eng.tok, model_cfg=eng.mcfg)
        if e2.is_driver:
            res["eager_tp2"] = [r.output_ids for r in e2.generate(prompts, greedy)]
            e2.stop_followers()
        else:
            e2.run_follower()
        torch.cuda.synchronize()
        res["ar_error"] = car.error() if car is not None else -1
        pd.destroy()
    except Exception:  # noqa: BLE001
        import traceback

        res["exc"] = traceback.format_exc()[-3000:]
    q.put(res)


def test_tp2_graphs_pipelined_match_tp1():
    """TP=2 on one GPU with decode and step graphs captured on both ranks and pipelined steps:
    greedy tokens equal the TP=1 eager engine's, the custom collectives never timed out, both
    ranks captured step graphs, the follower gathered its pipelined ids from its own samples,
    and after temperature sampling both ranks hold the same tokens."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_graph_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = sorted([q.get(timeout=300) for _ in range(2)], key=lambda r: r["rank"])
    for p in procs:
        p.join(timeout=60)
    print(results)
    for r in results:
        assert "exc" not in r, r["exc"]
        assert r["custom_ar"] and r["ar_error"] == 0, r
        assert r["async"] and r["use_graphs"] and r["mixed_graphs_ok"], r
        assert r["decode_graphs"] > 0 and r["step_graphs"] > 0, r
        assert r["gather_calls"] > 0, r
    drv, fol = results
    assert drv["out"] == drv["eager_tp2"], (drv["out"], drv["eager_tp2"])
    # against one rank: bf16 TP partial sums round differently; the peaky head keeps greedy
    # choices apart, so nearly every position agrees
    same = sum(a == b for o, r in zip(drv["out"], drv["ref"]) for a, b in zip(o, r))
    assert same >= 0.9 * sum(len(r) for r in drv["ref"]), (drv["out"], drv["ref"])
    assert all(len(o) == 12 for o in drv["hot"])
    assert fol["gathers"] > 0, fol
    assert drv["last_tok"] == fol["last_tok"]


def _ep_worker(rank, port, q):
    """Mixtral (mixtral-small: 8 experts, top-2) at TP = 2 with EXPERT parallelism: each rank
    holds 4 whole experts (its own routing slice), runs the grouped MFMA expert GEMMs
    (csrc/kernels/moe.hip) for the tokens routed to them, and the expert outputs meet in the
    all-reduce."""
    os.environ.update(RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    res = {"rank": rank}
    try:
        from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine, SamplingParams
        from nv_genai_amd.models.config import llama_config
        from nv_genai_amd.models.llama import LlamaModel
        from nv_genai_amd.parallel import dist as pd

        cfg = llama_config("mixtral-small")
        full = LlamaModel(cfg, "cpu", dtype=torch.bfloat16, pctx=pd.ParallelContext(), seed=7).state_dict()
        full["lm_head.weight"] = full["lm_head.weight"] * 40.0
        prompts = [[5, 6, 7, 8] * 30, [9, 10, 11] * 20]
        greedy = SamplingParams(temperature=0.0, max_tokens=10, ignore_eos=True, logprobs=True)
        ecfg = EngineConfig(model="mixtral-small", max_num_seqs=4, max_batched_tokens=1024, max_model_len=1024,
                            kv_cache_blocks=64, use_graphs=False)
        if rank == 0:
            e1 = LLMEngine(ecfg, device="cuda", pctx=pd.ParallelContext(), weights=full)
            res["ref"] = [(r.output_ids, r.logprobs) for r in e1.generate(prompts, greedy)]
            del e1
            torch.cuda.empty_cache()
        pctx = pd.init_distributed(tp_size=2, backend="gloo", device="cuda")
        eng = LLMEngine(ecfg, device="cuda", pctx=pctx, weights=full)
        res["ep"] = eng.model.expert_parallel
        res["experts"] = (eng.model.expert0, eng.model.n_experts)
        if eng.is_driver:
            res["out"] = [(r.output_ids, r.logprobs) for r in eng.generate(prompts, greedy)]
            eng.stop_followers()
        else:
            eng.run_follower()
        torch.cuda.synchronize()
        pd.destroy()
    except Exception:  # noqa: BLE001
        import traceback

        res["exc"] = traceback.format_exc()[-3000:]
    q.put(res)


def test_tp2_mixtral_expert_parallel_matches_tp1():
    """EP on the device: the two ranks hold experts [0, 4) and [4, 8); greedy tokens match one
    rank up to near-ties (test_engine_gpu._same_greedy_run)."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from test_engine_gpu import _same_greedy_run

    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ep_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = sorted([q.get(timeout=300) for _ in range(2)], key=lambda r: r["rank"])
    for p in procs:
        p.join(timeout=60)
    for r in results:
        assert "exc" not in r, r["exc"]
        assert r["ep"], r
    assert [r["experts"] for r in results] == [(0, 4), (4, 4)]
    drv = results[0]
    assert all(len(o) == 10 for o, _ in drv["out"])
    _same_greedy_run(drv["out"], drv["ref"])
