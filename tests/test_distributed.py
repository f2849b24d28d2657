"""Multi-process tests on CPU (gloo, world_size 2): tensor-parallel Llama matches TP=1
token-for-token, and the sharded vector index matches single-process search."""
import os
import socket

import pytest
import numpy as np
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tp_worker(rank, world, port, q, tp=2, pp=1, sp=False, model="llama-tiny", over=None, ekw=None):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine, SamplingParams
    from nv_genai_amd.models.config import llama_config
    from nv_genai_amd.models.llama import LlamaModel
    from nv_genai_amd.parallel import dist as pd

    single = pd.ParallelContext()
    cfg = llama_config(model, **(over or {}))
    full = LlamaModel(cfg, "cpu", pctx=single, seed=7).state_dict()
    ecfg = EngineConfig(model=model, max_num_seqs=4, max_batched_tokens=256, max_model_len=512,
                        kv_cache_blocks=32, sequence_parallel=sp, sp_min_tokens=16, **(ekw or {}))
    prompts = [[5, 6, 7, 8] * 20, [9, 10, 11] * 11]
    params = SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True)
    # fp32: a TP shard sums its partial products in a different order than one device, and
    # in bf16 that rounding can flip a near-tie greedy argmax of the random tiny model
    f32 = torch.float32
    ref = None
    if rank == 0:
        m1 = LlamaModel(cfg, "cpu", dtype=f32, pctx=single, weights=full)
        e1 = LLMEngine(ecfg, device="cpu", pctx=single, model=m1, model_cfg=cfg)
        ref = [r.output_ids for r in e1.generate(prompts, params)]
    pctx = pd.init_distributed(tp_size=tp, backend="gloo", device="cpu", pp_size=pp)
    eng = LLMEngine(ecfg, device="cpu", pctx=pctx, model_cfg=cfg,
                    model=LlamaModel(cfg, "cpu", dtype=f32, pctx=pctx, weights=full))
    if eng.is_driver:
        out = [r.output_ids for r in eng.generate(prompts, params)]
        eng.stop_followers()
        q.put((out, ref, eng.model.layer_lo, eng.model.layer_hi, eng.model.sp_steps))
    else:
        eng.run_follower()
    pd.destroy()


def _tp_pipeline_worker(rank, world, port, q):
    """TP=2 engine with pipelined steps: the driver launches step k + 1 before it reads step
    k's tokens, and every follower gathers those ids from its own sampled tokens."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine, SamplingParams
    from nv_genai_amd.models.config import llama_config
    from nv_genai_amd.models.llama import LlamaModel
    from nv_genai_amd.parallel import dist as pd

    single = pd.ParallelContext()
    cfg = llama_config("llama-tiny")
    full = LlamaModel(cfg, "cpu", pctx=single, seed=7).state_dict()
    ecfg = EngineConfig(model="llama-tiny", max_num_seqs=4, max_batched_tokens=256, max_model_len=512,
                        kv_cache_blocks=32)
    prompts = [[5, 6, 7, 8] * 20, [9, 10, 11] * 11, [3, 4] * 9]
    f32 = torch.float32
    greedy = SamplingParams(temperature=0.0, max_tokens=10, ignore_eos=True)
    hot = SamplingParams(temperature=0.9, top_p=0.9, max_tokens=10, ignore_eos=True, seed=11)
    ref = None
    if rank == 0:
        e1 = LLMEngine(ecfg, device="cpu", pctx=single, model_cfg=cfg,
                       model=LlamaModel(cfg, "cpu", dtype=f32, pctx=single, weights=full))
        ref = [r.output_ids for r in e1.generate(prompts, greedy)]
    pctx = pd.init_distributed(tp_size=2, backend="gloo", device="cpu")
    eng = LLMEngine(ecfg, device="cpu", pctx=pctx, model_cfg=cfg,
                    model=LlamaModel(cfg, "cpu", dtype=f32, pctx=pctx, weights=full))
    res = {"rank": rank, "async": eng.cfg.async_decode, "chan": type(eng._chan).__name__}
    if eng.is_driver:
        res["out"] = [r.output_ids for r in eng.generate(prompts, greedy)]
        res["hot"] = [r.output_ids for r in eng.generate(prompts, hot)]
        res["ref"] = ref
        res["unpipelined"] = eng.stats["unpipelined_steps"]
        res["pipelined"] = len(eng._host_steps)
        eng.stop_followers()
    else:
        eng.run_follower()
        res["gathers"] = eng._tp_gathers
    res["last_tok"] = eng.d_tok[:3].tolist()
    q.put(res)
    pd.destroy()


def test_tensor_parallel_steps_pipeline():
    """TP=2 over the shared-memory step channel keeps ``async_decode`` on: greedy tokens equal
    TP=1, most steps are launched before the previous step is read back, the follower applies
    the pipelined id gather to its own samples, and with temperature sampling both ranks end
    on the same sampled tokens (a follower that sampled differently would feed the all-reduces
    different embeddings and the driver's output would drift)."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_tp_pipeline_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda r: r["rank"])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    drv, fol = res
    assert drv["chan"] == "ShmStepChannel" and drv["async"] and fol["async"]
    assert drv["out"] == drv["ref"]
    assert all(len(o) == 10 for o in drv["hot"])
    assert drv["pipelined"] >= 10 and drv["unpipelined"] <= 4, drv
    assert fol["gathers"] >= 10, fol
    assert drv["last_tok"] == fol["last_tok"]


def test_tensor_parallel_matches_single():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_tp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out, ref, _, _, _ = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out == ref


def test_sequence_parallel_tp_matches_single():
    """TP=2 with sequence-parallel prefill (odd token counts exercise the row padding)."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_tp_worker, args=(r, world, port, q, 2, 1, True)) for r in range(world)]
    for p in procs:
        p.start()
    out, ref, _, _, sp_steps = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sp_steps >= 1
    assert out == ref


@pytest.mark.parametrize("model,over,sp", [
    ("mixtral-tiny", None, False),                    # 4 experts / 2 ranks: expert parallel
    ("mixtral-tiny", {"num_experts": 3}, False),       # 3 experts: each expert's FFN split
    ("starcoder2-tiny", None, True),                   # biases on rank 0, LayerNorm, window
    ("gemma-tiny", {"heads": 4, "kv_heads": 2}, False),
    ("gemma-tiny", {"heads": 4, "kv_heads": 1}, False),   # one KV head, replicated on both ranks
])
def test_tensor_parallel_families_match_single(model, over, sp):
    """Every decoder family at TP=2 generates the TP=1 tokens (Mixtral in both MoE sharding
    modes; StarCoder2 also with sequence-parallel prefill)."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_tp_worker, args=(r, world, port, q, 2, 1, sp, model, over))
             for r in range(world)]
    for p in procs:
        p.start()
    out, ref, _, _, _ = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out == ref


def test_tensor_parallel_graph_steps_match_single():
    """TP=2 with graph-layout prefill steps (run uncaptured on CPU: graph_eager): the
    followers rebuild the step's device layout from the broadcast payload (padded token
    rows included) and stay in lock-step with the driver's collectives."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ekw = {"mixed_graphs": True, "graph_eager": True, "graph_token_step": 32}
    procs = [ctx.Process(target=_tp_worker, args=(r, world, port, q, 2, 1, False, "llama-tiny",
                                                  {"head_dim": 128}, ekw)) for r in range(world)]
    for p in procs:
        p.start()
    out, ref, _, _, _ = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out == ref


@pytest.mark.parametrize("tp,pp", [(1, 2), (2, 2)])
def test_pipeline_parallel_matches_single(tp, pp):
    """Layer-split pipeline stages (optionally with TP inside each stage) generate the same
    tokens as one process holding the whole model."""
    world, port = tp * pp, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_tp_worker, args=(r, world, port, q, tp, pp)) for r in range(world)]
    for p in procs:
        p.start()
    out, ref, lo, hi, _ = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert (lo, hi) == (0, 1)  # the driver is stage 0 of the 2-layer tiny model
    assert out == ref


def _shard_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    from nv_genai_amd.index.flat import FlatIndex
    from nv_genai_amd.index.sharded import ShardedIndex
    from nv_genai_amd.parallel import dist as pd

    pctx = pd.init_distributed(tp_size=1, backend="gloo", device="cpu")
    g = torch.Generator().manual_seed(0)
    X = torch.randn(3000, 64, generator=g)
    Q = torch.randn(5, 64, generator=g)
    ids = torch.arange(3000) * 3
    sh = ShardedIndex(64, "cosine", "cpu", pctx=pctx)
    sh.add(X, ids)  # every rank passes the full set; each keeps its own stripe
    vals, out_ids = sh.search(Q if rank == 0 else torch.zeros(5, 64), 7)
    if rank == 0:
        full = FlatIndex(64, "cosine", "cpu")
        full.add(X, ids)
        rv, ri = full.search(Q, 7)
        # numpy, not tensors: a tensor's shared-memory fd dies with the worker before the parent reads it
        q.put((vals.numpy(), out_ids.numpy(), rv.numpy(), ri.numpy(), len(sh.local)))
    pd.destroy()


def test_sharded_index_matches_flat():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    vals, ids, rv, ri, nlocal = q.get(timeout=300)
    vals, ids, rv, ri = (torch.from_numpy(a) for a in (vals, ids, rv, ri))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert nlocal == 1500
    assert torch.allclose(vals, rv, atol=1e-5)
    assert torch.equal(ids, ri)


def _shard_snapshot_worker(rank, world, port, path, mode, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    from nv_genai_amd.index.sharded import ShardedIndex
    from nv_genai_amd.parallel import dist as pd

    pctx = pd.init_distributed(tp_size=1, backend="gloo", device="cpu")
    g = torch.Generator().manual_seed(1)
    X = torch.randn(1001, 32, generator=g)
    Q = torch.randn(4, 32, generator=g)
    if mode == "save":
        sh = ShardedIndex(32, "l2", "cpu", pctx=pctx)
        sh.add(X, torch.arange(1001) * 5)
        sh.remove([0, 5, 10])
        sh.save(path)
        sh.save(path)  # a second generation replaces the first; the old one is pruned
    else:
        sh = ShardedIndex.load(path, "cpu", pctx=pctx)
    vals, ids = sh.search(Q if rank == 0 else torch.zeros(4, 32), 6)
    n = len(sh)
    if rank == 0:
        q.put((vals.numpy(), ids.numpy(), n))
    pd.destroy()


def _run_world(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, *args, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return tuple(torch.from_numpy(a) if isinstance(a, np.ndarray) else a for a in out)


def test_sharded_index_snapshot_restore_and_restripe(tmp_path):
    """Sharded snapshot: per-rank safetensors shards + an atomically published
    manifest; restoring on the same world size and on a different one gives the same search."""
    import json

    path = str(tmp_path / "idx")
    v0, i0, n0 = _run_world(_shard_snapshot_worker, 2, path, "save")
    man = json.loads((tmp_path / "idx" / "manifest.json").read_text())
    assert man["world"] == 2 and man["total"] == n0 == 998
    gens = [d.name for d in (tmp_path / "idx").iterdir() if d.name.startswith("gen-")]
    assert len(gens) == 2 and man["generation"] in gens  # new + one kept
    v1, i1, n1 = _run_world(_shard_snapshot_worker, 2, path, "load")
    assert n1 == 998 and torch.equal(i0, i1) and torch.allclose(v0, v1, atol=1e-5)
    v3, i3, n3 = _run_world(_shard_snapshot_worker, 3, path, "load")  # re-striped to 3 ranks
    assert n3 == 998 and torch.equal(i0, i3) and torch.allclose(v0, v3, atol=1e-4)
    assert not bool((i0 == 0).any() | (i0 == 5).any() | (i0 == 10).any())


def test_all_reduce_routes_to_registered_custom_all_reduce():
    """comm.all_reduce takes a group's custom all-reduce when the tensor is eligible and
    falls back to the process group otherwise."""
    from nv_genai_amd.parallel import comm

    class FakeCAR:
        def __init__(self):
            self.calls = 0

        def eligible(self, x):
            return x.numel() <= 4

        def all_reduce(self, x):
            self.calls += 1
            return x.mul_(2)

    group = object()
    car = FakeCAR()
    comm.register_custom_all_reduce(group, car)
    try:
        assert comm.custom_all_reduce_for(group) is car
        x = torch.ones(4)
        comm.all_reduce(x, group)
        assert car.calls == 1 and torch.equal(x, torch.full((4,), 2.0))
    finally:
        comm.register_custom_all_reduce(group, None)
    assert comm.custom_all_reduce_for(group) is None


def test_agent_benchmark_tp2_sharded_index(tmp_path):
    """benchmarks/agent_tp.py on CPU (gloo): one TP=2 replica whose sharded-index searches
    travel the engine's step channel (broadcast_command + EngineService.call) between LLM
    steps; every scripted agent finishes and the JSON line reports it."""
    import json
    import subprocess
    import sys

    port = _free_port()
    out = tmp_path / "agent.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", "benchmarks/agent_tp.py",
           "--model", "llama-tiny", "--embed-model", "encoder-tiny", "--index-size", "5000",
           "--queries", "6", "--warmup", "1", "--concurrency", "3", "--plan-tokens", "4",
           "--extract-tokens", "4", "--answer-tokens", "6", "--max-num-seqs", "8", "--out", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=os.getcwd()))
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    res = json.loads(out.read_text())
    assert res["parallelism"] == "tp2" and res["queries"] == 6 and res["value"] > 0
    assert res["searches_per_s"] > 0 and res["llm_calls_per_s"] > 0


def _sharded_ids_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from nv_genai_amd.index.sharded import ShardedIndex
    from nv_genai_amd.parallel import dist as pd

    pd.init_distributed()
    idx = ShardedIndex(16, "cosine", "cpu")
    idx.add_random(101, seed=3)
    ids = idx.local.ids[: idx.local.n].tolist()
    q.put((rank, ids, len(idx)))
    pd.destroy()


def test_sharded_random_ids_are_global():
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_sharded_ids_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(60)
    all_ids = sorted(i for _, ids, _ in got for i in ids)
    assert all_ids == list(range(101)) and all(n == 101 for _, _, n in got)


def _step_channel_fallback_worker(rank, world, port, q):
    import os

    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import numpy as np

    from nv_genai_amd.parallel import dist as pd
    from nv_genai_amd.parallel import step_channel as sc

    pctx = pd.init_distributed(tp_size=2, backend="gloo", device="cpu")
    if rank == 1:   # this follower cannot open the driver's segment (as on another host)
        real = sc.rt.ShmChannel

        def failing(name, create, *a):
            if not create:
                raise OSError("no such segment")
            return real(name, create, *a)

        sc.rt = type("RT", (), {"ShmChannel": staticmethod(failing)})
    chan = sc.create(pctx, 4096, transport="shm")
    msg = np.arange(100, dtype=np.int64)
    if rank == 0:
        chan.send(msg)
        got = None
    else:
        got = chan.recv().view(np.int64).tolist()
    q.put({"rank": rank, "chan": type(chan).__name__, "got": got})
    pd.destroy()


def test_step_channel_falls_back_when_a_follower_cannot_attach():
    """A replica whose follower cannot open the shared-memory segment (ranks on different hosts
    that looked alike) agrees on the broadcast channel on every rank instead of hanging."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_step_channel_fallback_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r["rank"])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r["chan"] for r in res] == ["DistStepChannel", "DistStepChannel"]
    assert res[1]["got"] == list(range(100))
