"""World-size 4 and 8 correctness on CPU (gloo), the layouts the 8-GPU node runs:

* TP=8 with Llama-3-70B's head ratio (64 q : 8 kv heads -> 8 q heads and 1 KV head per rank,
  the north-star layout of BASELINE.json configs[3]); layers and widths shrunk;
* TP=4, and TP=4 x PP=2 over 8 ranks;
* TP=2 x DP=4 replicas (each replica generates on its own);
* the sharded index at world 8 against one flat index;
* ``bench.py --gpus 8`` self-launching 8 ranks for the agent workload (TP=8 + 8-way sharded
  index) and for TP=2 x 4 RAG replicas with sharded indexes;
* the custom all-reduce's algorithm choice (two-shot above the threshold once W > 2) through
  the Python routing that the model's all-reduces take.

Every rank pins torch to one intra-op thread: 8 ranks share this container's 8 CPUs.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


HEAD_70B = {"hidden": 256, "heads": 64, "kv_heads": 8, "head_dim": 16, "ffn": 512}
TINY_8Q4KV = {"heads": 8, "kv_heads": 4, "head_dim": 32}


def _tp_worker(rank, world, port, tp, pp, over, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine, SamplingParams
    from nv_genai_amd.models.config import llama_config
    from nv_genai_amd.models.llama import LlamaModel
    from nv_genai_amd.parallel import dist as pd

    single = pd.ParallelContext()
    cfg = llama_config("llama-tiny", **over)
    full = LlamaModel(cfg, "cpu", pctx=single, seed=11).state_dict()
    ecfg = EngineConfig(model="llama-tiny", max_num_seqs=4, max_batched_tokens=256, max_model_len=512,
                        kv_cache_blocks=32)
    prompts = [[5, 6, 7, 8] * 20, [9, 10, 11] * 11, [3] * 70]
    params = SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True, logprobs=True)
    f32 = torch.float32
    pctx = pd.init_distributed(tp_size=tp, backend="gloo", device="cpu", pp_size=pp)
    ref = None
    if pctx.tp_rank == 0 and pctx.pp_rank == 0:
        # every replica's driver computes the single-process answer for its own prompts
        m1 = LlamaModel(cfg, "cpu", dtype=f32, pctx=single, weights=full)
        e1 = LLMEngine(ecfg, device="cpu", pctx=single, model=m1, model_cfg=cfg)
        ref = [(r.output_ids, r.logprobs) for r in e1.generate(prompts, params)]
    model = LlamaModel(cfg, "cpu", dtype=f32, pctx=pctx, weights=full)
    eng = LLMEngine(ecfg, device="cpu", pctx=pctx, model_cfg=cfg, model=model)
    if eng.is_driver:
        out = [(r.output_ids, r.logprobs) for r in eng.generate(prompts, params)]
        eng.stop_followers()
        q.put((pctx.dp_rank, out, ref, model.hq, model.hkv))
    else:
        eng.run_follower()
    pd.destroy()


def _run(world, tp, pp, over, n_results):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tp_worker, args=(r, world, port, tp, pp, over, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=600) for _ in range(n_results)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return got


def _check(gens):
    """Same greedy tokens as TP=1, and the same log-probabilities of them (the sampled
    token's log-softmax of the full-vocabulary logits, all-gathered over the TP ranks)."""
    for _, out, ref, _, _ in gens:
        assert [o for o, _ in out] == [o for o, _ in ref]
        for (_, lp), (_, lp_ref) in zip(out, ref):
            assert len(lp) == len(lp_ref) > 0
            assert torch.allclose(torch.tensor(lp), torch.tensor(lp_ref), atol=1e-4, rtol=1e-4)
    return gens


def test_tp8_70b_head_ratio_matches_single():
    """TP=8 with 64 q : 8 kv heads: each rank holds 8 q heads and exactly 1 KV head."""
    gens = _check(_run(8, 8, 1, HEAD_70B, 1))
    assert [(hq, hkv) for _, _, _, hq, hkv in gens] == [(8, 1)]


def test_tp8_with_two_kv_heads_replicates_them():
    """TP=8 over a model with 2 KV heads: each KV head lives on 4 ranks (those whose query
    heads attend to it); tokens and log-probs still match one process."""
    gens = _check(_run(8, 8, 1, {"heads": 8, "kv_heads": 2, "head_dim": 32}, 1))
    assert [(hq, hkv) for _, _, _, hq, hkv in gens] == [(1, 1)]


def test_tp4_matches_single():
    gens = _check(_run(4, 4, 1, TINY_8Q4KV, 1))
    assert [(hq, hkv) for _, _, _, hq, hkv in gens] == [(2, 1)]


def test_tp4_pp2_world8_matches_single():
    gens = _check(_run(8, 4, 2, TINY_8Q4KV, 1))
    assert len(gens) == 1


def test_tp2_dp4_world8_replicas_match_single():
    """Four independent TP=2 replicas on one 8-rank job: every driver matches TP=1."""
    gens = _check(_run(8, 2, 1, TINY_8Q4KV, 4))
    assert sorted(g[0] for g in gens) == [0, 1, 2, 3]


# ---------------------------------------------------------------- sharded index at world 8
def _shard8_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from nv_genai_amd.index.flat import FlatIndex
    from nv_genai_amd.index.sharded import ShardedIndex
    from nv_genai_amd.parallel import dist as pd

    pctx = pd.init_distributed(tp_size=1, backend="gloo", device="cpu")
    g = torch.Generator().manual_seed(5)
    X = torch.randn(4003, 48, generator=g)
    Q = torch.randn(9, 48, generator=g)
    ids = torch.arange(4003) * 7 + 1
    sh = ShardedIndex(48, "cosine", "cpu", pctx=pctx)
    sh.add(X, ids)
    vals, out_ids = sh.search(Q if rank == 0 else torch.zeros(9, 48), 10)
    n = len(sh)
    if rank == 0:
        full = FlatIndex(48, "cosine", "cpu")
        full.add(X, ids)
        rv, ri = full.search(Q, 10)
        q.put((vals.numpy(), out_ids.numpy(), rv.numpy(), ri.numpy(), n, len(sh.local)))
    pd.destroy()


def test_sharded_index_world8_matches_flat():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard8_worker, args=(r, 8, port, q)) for r in range(8)]
    for p in procs:
        p.start()
    vals, ids, rv, ri, n, nlocal = q.get(timeout=300)
    vals, ids, rv, ri = (torch.from_numpy(a) for a in (vals, ids, rv, ri))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert n == 4003 and nlocal == 501   # rows 0, 8, 16, ... of 4003
    assert torch.allclose(vals, rv, atol=1e-5)
    assert torch.equal(ids, ri)


# ---------------------------------------------------------------- bench.py at 8 ranks
def _bench(args, timeout=900):
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py"] + args, cwd=ROOT, capture_output=True, text=True,
                       timeout=timeout, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


def test_bench_self_launch_agent_tp8_sharded_index():
    """``python bench.py --gpus 8 --workload agent``: bench.py starts torch.distributed.run
    itself; one TP=8 replica of the 64 q : 8 kv-head tiny model (``llama70b-tiny``: 1 KV head
    per rank, as Llama-3-70B at TP=8) and an 8-way sharded index."""
    res = _bench(["--gpus", "8", "--workload", "agent", "--steps", "1", "--warmup", "0",
                  "--model", "llama70b-tiny", "--embed-model", "encoder-tiny", "--index-size", "8000",
                  "--concurrency", "2", "--max-tokens", "4"])
    assert res["n_gpus"] == 8 and res["world_size"] == 8 and res["config"]["parallelism"] == "tp8"
    assert res["config"]["sharded_index"] and res["value"] > 0 and res["searches_per_s"] > 0


def test_bench_self_launch_rag_tp2_dp4_sharded():
    res = _bench(["--gpus", "8", "--tp", "2", "--sharded-index", "--steps", "1", "--warmup", "1",
                  "--model", "llama-tiny", "--embed-model", "encoder-tiny", "--index-size", "4000",
                  "--concurrency", "2", "--max-tokens", "3"])
    assert res["n_gpus"] == 8 and res["config"]["parallelism"] == "dp4xtp2"
    assert res["config"]["sharded_index"] and len(res["per_replica_qps"]) == 4
    assert res["config"]["global_batch"] == 8
    assert abs(res["value"] - 8 / (res["ms_per_step"] / 1000)) / res["value"] < 0.01


def test_bench_gpus_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="1", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2"], cwd=ROOT, capture_output=True,
                       text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)


# ---------------------------------------------------------------- custom all-reduce routing
def test_custom_all_reduce_algo_choice():
    from nv_genai_amd.parallel.custom_ar import ALGO_ONE_SHOT, ALGO_TWO_SHOT, choose_algo

    assert choose_algo(16 << 10, 8) == ALGO_ONE_SHOT          # 70B decode message (1 token)
    assert choose_algo(4 << 20, 8) == ALGO_TWO_SHOT           # prefill-sized message
    assert choose_algo(4 << 20, 2) == ALGO_ONE_SHOT           # W = 2: two-shot saves nothing
    assert choose_algo(512 << 10, 4) == ALGO_ONE_SHOT         # at the threshold
    assert choose_algo((512 << 10) + 16, 4) == ALGO_TWO_SHOT


def test_custom_all_reduce_auto_routes_two_shot_through_comm():
    """comm.all_reduce -> CustomAllReduce.all_reduce(AUTO) hands the kernel an explicit
    two-shot for a large message at W = 8 and one-shot for a decode-sized one."""
    from nv_genai_amd.parallel import comm
    from nv_genai_amd.parallel.custom_ar import ALGO_ONE_SHOT, ALGO_TWO_SHOT, CustomAllReduce, \
        TWO_SHOT_THRESHOLD_BYTES

    class Impl:
        def __init__(self):
            self.algos = []

        def all_reduce(self, x, out, algo):
            self.algos.append(algo)
            out.copy_(x * 8)

    car = object.__new__(CustomAllReduce)
    car.world, car.enabled, car.capacity = 8, True, 64 << 20
    car.two_shot_threshold = TWO_SHOT_THRESHOLD_BYTES
    car.algo_counts = {ALGO_ONE_SHOT: 0, ALGO_TWO_SHOT: 0}
    car.impl = Impl()
    car.eligible = lambda x: True      # CPU tensors stand in for device ones
    group = object()
    comm.register_custom_all_reduce(group, car)
    try:
        big = torch.ones(1 << 20, dtype=torch.bfloat16)      # 2 MiB
        small = torch.ones(8192, dtype=torch.bfloat16)       # 16 KiB: one 70B decode token
        comm.all_reduce(big, group)
        comm.all_reduce(small, group)
    finally:
        comm.register_custom_all_reduce(group, None)
    assert car.impl.algos == [ALGO_TWO_SHOT, ALGO_ONE_SHOT]
    assert car.algo_counts == {ALGO_ONE_SHOT: 1, ALGO_TWO_SHOT: 1}
    assert float(big[0]) == 8.0 and float(small[0]) == 8.0


def _shard_payload_worker(rank, world, port, q):
    """The search command's path: the driver's query block arrives as channel payload bytes
    (query_payload -> queries_from_payload), no broadcast; ids past 2^31 and short shards
    (-1 padding) survive the packed int32 gather."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from nv_genai_amd.index.flat import FlatIndex
    from nv_genai_amd.index.sharded import ShardedIndex
    from nv_genai_amd.parallel import dist as pd

    pctx = pd.init_distributed(tp_size=1, backend="gloo", device="cpu")
    g = torch.Generator().manual_seed(9)
    X = torch.randn(21, 32, generator=g)          # 21 rows over 4 ranks: shards of 6/5/5/5 < k
    Q = torch.randn(3, 32, generator=g)
    ids = torch.arange(21, dtype=torch.int64) * 3_000_000_019 + 5    # up to 6e10 > 2^31
    sh = ShardedIndex(32, "cosine", "cpu", pctx=pctx)
    sh.add(X, ids)
    payload = sh.query_payload(Q)                 # what the driver puts in the command
    qq = sh.queries_from_payload(3, payload.view(np.uint8).reshape(-1))
    vals, out_ids = sh.search(qq, 8, have_queries=True)
    if rank == 0:
        full = FlatIndex(32, "cosine", "cpu")
        full.add(X, ids)
        rv, ri = full.search(Q, 8)
        q.put((vals.numpy(), out_ids.numpy(), rv.numpy(), ri.numpy(), dict(sh.stats)))
    pd.destroy()


def test_sharded_search_from_command_payload_packed_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_payload_worker, args=(r, 4, port, q)) for r in range(4)]
    for p in procs:
        p.start()
    vals, ids, rv, ri, st = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert torch.allclose(torch.from_numpy(vals), torch.from_numpy(rv), atol=1e-5)
    assert torch.equal(torch.from_numpy(ids), torch.from_numpy(ri))
    assert st["broadcasts"] == 0 and st["pg_gathers"] == 1 and st["searches"] == 1
