"""TP = 8 rehearsal on the box's one MI355X: eight ranks share cuda:0 and run the engine path
a TP = 8 node runs (BASELINE.json configs[3], Llama-3-70B at TP = 8; the reference's
``tensor_para_size`` / ``enable_custom_all_reduce``,
experimental/fm-asr-streaming-rag/nim/configs/mistral-7b.yaml:32-36):

* the 70B attention layout at its real head_dim (``llama70b-small``: 64 q : 8 kv heads of 128,
  so each rank holds 8 q heads and one KV head, and a q/k/v shard of 1280 columns);
* decode graphs and prefill / mixed step graphs captured on all eight ranks;
* pipelined steps over the shared-memory step channel with seven readers;
* step messages large enough (hidden 2048: 1 MiB at 256 tokens) that the custom all-reduce
  takes its two-shot form inside captured graphs, the fused all-reduce + residual + RMSNorm
  for decode rows, and the W = 8 IPC all-gather of the vocab-parallel logits;
* the same run with ``NGA_CUSTOM_AR=0``: every collective over gloo, graphs off (a graph may
  hold only IPC collectives), and the same tokens.

Tokens must equal a synchronous (unpipelined) W = 8 run with the same graphs, and match an eager
W = 8 run (no bucket padding, so the library GEMMs may pick other kernels) and TP = 1 (bf16
partial sums round differently) up to near-tie divergences (test_engine_gpu._same_greedy_run).
Every all-reduce / all-gather meets its peers in time (sticky timeout code 0).

Found by this rehearsal: with every rank's grid at the 80-block cap, the eight ranks' spinning
all-reduce blocks were not all resident at once beside the engine's other kernels and the
barriers timed out (code 1-5, garbage sums ever after); ranks that share a device now split the
cap (``CustomAllReduce.ranks_per_device``). Host groups are gloo: RCCL refuses two ranks on one
device. Each rank limits itself to two HIP hardware queues (16 over the eight processes).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

WORLD = 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, q, custom_ar, over=None):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(WORLD), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), GPU_MAX_HW_QUEUES="2", NGA_CUSTOM_AR="1" if custom_ar else "0",
                      OMP_NUM_THREADS="1", NGA_NUMA_BIND="0")
    torch.set_num_threads(1)
    res = {"rank": rank}
    try:
        import dataclasses
        import time

        from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine, SamplingParams
        from nv_genai_amd.models.config import llama_config
        from nv_genai_amd.models.llama import LlamaModel
        from nv_genai_amd.parallel import comm
        from nv_genai_amd.parallel import custom_ar as cal
        from nv_genai_amd.parallel import dist as pd

        cfg = llama_config("llama70b-small")
        full = LlamaModel(cfg, "cpu", dtype=torch.bfloat16, pctx=pd.ParallelContext(), seed=5).state_dict()
        full["lm_head.weight"] = full["lm_head.weight"] * 40.0   # peaky logits: no greedy near-ties
        # 120 + 60 + 140 + 90 prompt tokens: a 410-token prefill step (bucket 512: a 2 MiB
        # all-reduce), then decode steps of 4 rows (16 KiB: one-shot, fused add + RMSNorm)
        prompts = [[5, 6, 7, 8] * 30, [9, 10, 11] * 20, [12, 13] * 70, [21, 22, 23] * 30]
        greedy = SamplingParams(temperature=0.0, max_tokens=16, ignore_eos=True, logprobs=True)
        hot = SamplingParams(temperature=0.8, top_p=0.9, max_tokens=12, ignore_eos=True, seed=3)
        ecfg = EngineConfig(model="llama70b-small", max_num_seqs=4, max_batched_tokens=1024, max_model_len=1024,
                            kv_cache_blocks=64, use_graphs=True, mixed_graphs=True, graph_token_step=128,
                            mixed_prefill_tokens=512, graph_batch_sizes=(1, 2, 4))
        if over:
            ecfg = dataclasses.replace(ecfg, **over)
        if rank == 0:
            e1 = LLMEngine(dataclasses.replace(ecfg, use_graphs=False, mixed_graphs=False), device="cuda",
                           pctx=pd.ParallelContext(), weights=full)
            res["ref"] = [(r.output_ids, r.logprobs) for r in e1.generate(prompts, greedy)]
            del e1
            torch.cuda.empty_cache()
        pctx = pd.init_distributed(tp_size=WORLD, backend="gloo", device="cuda")
        car = comm.custom_all_reduce_for(pctx.tp_group)
        res["custom_ar"] = car is not None and car.enabled
        t0 = time.time()
        eng = LLMEngine(ecfg, device="cuda", pctx=pctx, weights=full)
        res["setup_s"] = round(time.time() - t0, 1)
        res["hq_hkv"] = (eng.model.hq, eng.model.hkv)
        res["chan"] = type(eng._chan).__name__
        res["async"] = eng.cfg.async_decode
        res["use_graphs"] = eng.cfg.use_graphs
        res["mixed_graphs_ok"] = eng._mg_ok
        torch.cuda.synchronize()
        res["ar_error_init"] = car.error() if car is not None else 0
        if eng.is_driver:
            res["out"] = [(r.output_ids, r.logprobs) for r in eng.generate(prompts, greedy)]
            res["hot"] = [r.output_ids for r in eng.generate(prompts, hot)]
            res["unpipelined"] = eng.stats["unpipelined_steps"]
            res["graph_steps"] = eng.stats["graph_steps"]
            eng.stop_followers()
        else:
            eng.run_follower()
            res["gathers"] = eng._tp_gathers
            res["follower"] = eng.follower_stats()
        torch.cuda.synchronize()
        res["ar_error_mid"] = car.error() if car is not None else 0
        res["decode_graphs"] = len(eng.graphs)
        res["step_graphs"] = len(eng.mgraphs)
        res["last_tok"] = eng.d_tok[:4].tolist()
        st = cal.status()
        res["algo_counts"] = st.get("algo_counts")
        res["max_blocks"] = st.get("max_blocks")
        res["gather_calls"] = car.gather_count if car is not None else 0
        # the same replica with the same graphs but synchronous steps (the pipelining is the only
        # difference: tokens must be identical), then eager and synchronous (no bucket padding:
        # the library GEMMs may pick other kernels at the unpadded row counts, so near-tied
        # greedy choices can differ; >= 90 % of positions agree)
        for key, o in (("sync", dict(async_decode=False)),
                       ("eager", dict(use_graphs=False, mixed_graphs=False, async_decode=False))):
            e2 = LLMEngine(dataclasses.replace(ecfg, **o), device="cuda", pctx=pctx, model=eng.model,
                           tokenizer=eng.tok, model_cfg=eng.mcfg)
            if e2.is_driver:
                res[key] = [(r.output_ids, r.logprobs) for r in e2.generate(prompts, greedy)]
                e2.stop_followers()
            else:
                e2.run_follower()
            del e2
        torch.cuda.synchronize()
        res["ar_error"] = car.error() if car is not None else 0
        pd.destroy()
    except Exception:  # noqa: BLE001
        import traceback

        res["exc"] = traceback.format_exc()[-3000:]
    q.put(res)


def _run(custom_ar: bool, over=None, check=True):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, port, q, custom_ar, over)) for r in range(WORLD)]
    for p in procs:
        p.start()
    try:
        results = sorted([q.get(timeout=400) for _ in range(WORLD)], key=lambda r: r["rank"])
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    print(results)
    for r in results:
        if check:
            assert "exc" not in r, (r["rank"], r["exc"])
    return results


def _check_tokens(results):
    from test_engine_gpu import _same_greedy_run

    drv = results[0]
    assert drv["hq_hkv"] == (8, 1), drv
    assert all(len(o) == 16 for o, _ in drv["out"])
    # pipelined vs synchronous steps over the same graphs: identical tokens
    assert [o for o, _ in drv["out"]] == [o for o, _ in drv["sync"]], (drv["out"], drv["sync"])
    # vs eager W = 8 and vs TP = 1: equal first tokens, log-probs close until a divergence, and
    # a divergence only at a near-tie (random weights: bucket padding or another partial-sum
    # order can flip an exact tie, after which a greedy sequence follows another path)
    _same_greedy_run(drv["out"], drv["eager"])
    _same_greedy_run(drv["out"], drv["ref"])
    assert all(len(o) == 12 for o in drv["hot"])
    # after temperature sampling every rank holds the driver's tokens
    assert all(r["last_tok"] == drv["last_tok"] for r in results), [r["last_tok"] for r in results]


def test_tp8_graphs_pipelined_two_shot_on_one_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    results = _run(custom_ar=True)
    _check_tokens(results)
    drv = results[0]
    assert drv["unpipelined"] == 0 and drv["graph_steps"] > 0, drv
    for r in results:
        assert r["chan"] == "ShmStepChannel" and r["async"], r
        assert r["custom_ar"] and r["ar_error"] == 0, r
        assert r["use_graphs"] and r["mixed_graphs_ok"], r
        assert r["decode_graphs"] > 0 and r["step_graphs"] > 0, r
        assert r["algo_counts"]["two_shot"] > 0 and r["algo_counts"]["one_shot"] > 0, r
        assert r["gather_calls"] > 0, r
    for r in results[1:]:
        assert r["gathers"] > 0, r
        f = r["follower"]
        assert f["channel"]["messages"] > 0 and f["channel"]["lat_n"] > 0, f


def test_tp8_without_custom_all_reduce_falls_back():
    """NGA_CUSTOM_AR=0: all-reduces and the logits gather go over the host group, so graphs
    are off on every rank (none may capture a non-IPC collective) and steps run eagerly, with
    the same greedy tokens."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    results = _run(custom_ar=False)
    _check_tokens(results)
    for r in results:
        assert not r["custom_ar"], r
        assert not r["use_graphs"] and not r["mixed_graphs_ok"], r
        assert r["decode_graphs"] == 0 and r["step_graphs"] == 0, r


def _shard_worker(rank, port, q):
    """One rank of an 8-way sharded index on the shared GPU: the query block arrives as the
    search command's payload bytes, the (score, id) lists meet in ONE IPC all-gather."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(WORLD), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), GPU_MAX_HW_QUEUES="2", OMP_NUM_THREADS="1", NGA_NUMA_BIND="0")
    torch.set_num_threads(1)
    res = {"rank": rank}
    try:
        from nv_genai_amd.index.flat import FlatIndex
        from nv_genai_amd.index.sharded import ShardedIndex
        from nv_genai_amd.parallel import dist as pd

        pctx = pd.init_distributed(tp_size=1, backend="gloo", device="cuda")
        dev = torch.device("cuda", 0)
        g = torch.Generator().manual_seed(21)
        X = torch.randn(20_003, 1024, generator=g)
        Q = torch.randn(9, 1024, generator=g)
        ids = torch.arange(20_003, dtype=torch.int64) * 7 + 3
        sh = ShardedIndex(1024, "cosine", "cuda", pctx=pctx, capacity=20_003 // WORLD + 1)
        sh.add(X, ids)
        payload = sh.query_payload(Q)
        vals, out_ids = sh.search(sh.queries_from_payload(9, payload.view("uint8").reshape(-1)), 10,
                                  have_queries=True)
        torch.cuda.synchronize()
        res["stats"] = dict(sh.stats)
        res["ipc"] = sh._car is not None
        if rank == 0:
            full = FlatIndex(1024, "cosine", "cuda", capacity=20_003)
            full.add(X, ids)
            rv, ri = full.search(Q.to(dev), 10)
            res["vals_diff"] = float((vals - rv).abs().max())
            res["ids_equal"] = bool(torch.equal(out_ids.cpu(), ri.cpu()))
        res["error"] = sh._car.error() if sh._car is not None else -1
        pd.destroy()
    except Exception:  # noqa: BLE001
        import traceback

        res["exc"] = traceback.format_exc()[-3000:]
    q.put(res)


def test_sharded_index_ipc_gather_matches_flat_eight_ranks():
    """CC7/CC8 on the device at W = 8: no broadcast (queries from the command payload), one
    IPC all-gather of the packed (score, id) rows, merged top-10 equal to one flat index."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_shard_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    try:
        results = sorted([q.get(timeout=300) for _ in range(WORLD)], key=lambda r: r["rank"])
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in results:
        assert "exc" not in r, (r["rank"], r["exc"])
        assert r["ipc"] and r["error"] == 0, r
        assert r["stats"]["broadcasts"] == 0 and r["stats"]["ipc_gathers"] == 1 and r["stats"]["pg_gathers"] == 0, r
    r0 = results[0]
    assert r0["ids_equal"] and r0["vals_diff"] < 1e-3, r0
