"""Custom IPC all-reduce (csrc/kernels/custom_ar.hip) on the GPU box.

The box has ONE MI355X, so the two ranks share cuda:0: each process exports its uncached
Signal+staging allocation with hipIpcGetMemHandle and maps the other's, exactly as across
xGMI peers (what this cannot show is cross-GPU cache coherence — the start-up self-test
against RCCL covers that on a real TP group). Handles and the reference sums go over gloo.

Expected values: each rank's input is a deterministic function of (rank, case), so every
process recomputes all inputs and the exact fp32 sum in rank order 0..W-1 — the kernel's
own summation order — and the result must match bit for bit.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

WORLD = 2
CASES = [  # (numel, dtype, algo)
    (8, torch.bfloat16, 1),
    (8192, torch.bfloat16, 0),
    (8192 * 64, torch.bfloat16, 1),
    (8192 * 64, torch.bfloat16, 2),
    (8192 * 256 + 8, torch.bfloat16, 2),   # chunk does not divide evenly
    (3 * 1024 * 1024, torch.bfloat16, 0),  # auto -> two-shot
    (4096, torch.float32, 1),
    (1 << 20, torch.float32, 2),
]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inp(rank, ci, n, dtype):
    g = torch.Generator().manual_seed(7919 * ci + rank)
    return torch.randn(n, generator=g).to(dtype)


def _expect(ci, n, dtype, world=WORLD):
    acc = torch.zeros(n, dtype=torch.float32)
    for r in range(world):
        acc = acc + _inp(r, ci, n, dtype).float()
    return acc.to(dtype)


CASES4 = [  # 4 ranks: the auto choice (one-shot small, two-shot above 512 KiB) and forced two-shot
    (8192, torch.bfloat16, 0),
    (3 * 1024 * 1024, torch.bfloat16, 0),
    (8192 * 256 + 8, torch.bfloat16, 2),
    (1 << 20, torch.float32, 0),
]


def _worker4(rank, port, q, world=4):
    """Four ranks on the one GPU: exact sums and the algorithm the Python routing picked."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import torch.distributed as dist

    from nv_genai_amd.parallel.custom_ar import CustomAllReduce

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {"rank": rank}
    try:
        car = CustomAllReduce(None, capacity_mb=16, timeout_s=10.0)
        res["self_test"] = car.enabled
        bad = []
        for ci, (n, dt, algo) in enumerate(CASES4):
            x = _inp(rank, ci, n, dt).cuda()
            out = car.all_reduce(x, out=torch.empty_like(x), algo=algo)
            torch.cuda.synchronize()
            if not torch.equal(out.cpu(), _expect(ci, n, dt, world)):
                bad.append(ci)
        res["bad"] = bad
        res["algo_counts"] = dict(car.algo_counts)
        res["error"] = car.error()
    except Exception as e:  # noqa: BLE001
        res["exc"] = repr(e)
    q.put(res)
    dist.destroy_process_group()


def test_custom_all_reduce_four_ranks_two_shot_auto():
    """W = 4 takes the two-shot path for messages above 512 KiB (choose_algo, resolved in
    Python) and the sums stay bit-exact in rank order."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker4, args=(r, port, q)) for r in range(4)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert "exc" not in r, r
        assert r["self_test"] and r["bad"] == [] and r["error"] == 0, r
        # self-test: one-shot + two-shot + auto(1 MiB -> two-shot); cases: auto small -> one,
        # auto 6 MiB -> two, forced two, auto 4 MiB fp32 -> two
        assert r["algo_counts"] == {1: 2, 2: 5}, r["algo_counts"]


def _worker(rank, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(WORLD), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import torch.distributed as dist

    from nv_genai_amd.parallel.custom_ar import CustomAllReduce

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    res = {"rank": rank}
    try:
        car = CustomAllReduce(None, capacity_mb=16, timeout_s=10.0)
        res["self_test"] = car.enabled
        bad = []
        for ci, (n, dt, algo) in enumerate(CASES):
            x = _inp(rank, ci, n, dt).cuda()
            out = car.all_reduce(x, out=torch.empty_like(x), algo=algo)
            inplace = car.all_reduce(x.clone(), algo=algo)
            torch.cuda.synchronize()
            exp = _expect(ci, n, dt)
            if not torch.equal(out.cpu(), exp) or not torch.equal(inplace.cpu(), exp):
                bad.append((ci, float((out.cpu().float() - exp.float()).abs().max())))
        res["bad"] = bad
        # fused epilogue: resid += all_reduce(x); out = rmsnorm(resid) * w
        fused_bad = []
        for ci, (rows, H) in enumerate(((1, 4096), (7, 4096), (64, 8192), (200, 1024))):
            x = _inp(rank, 50 + ci, rows * H, torch.bfloat16).view(rows, H).cuda()
            resid0 = _inp(99, 60 + ci, rows * H, torch.bfloat16).view(rows, H)
            w = (_inp(98, 70 + ci, H, torch.bfloat16).float().abs() + 0.5).to(torch.bfloat16)
            resid = resid0.clone().cuda()
            out = car.all_reduce_add_rmsnorm(x, resid, w.cuda(), 1e-5)
            torch.cuda.synchronize()
            s_ = _expect(50 + ci, rows * H, torch.bfloat16).view(rows, H)
            r_exp = (resid0.float() + s_.float()).to(torch.bfloat16)
            xf = r_exp.float()
            o_exp = (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float())
            if not torch.equal(resid.cpu(), r_exp) or (out.cpu().float() - o_exp).abs().max() > 0.02 * o_exp.abs().max():
                fused_bad.append(ci)
        res["fused_bad"] = fused_bad
        # hipGraph: 3 all-reduces captured once, replayed twice with new inputs
        xs = [torch.empty(8192 * 16, dtype=torch.bfloat16, device="cuda") for _ in range(3)]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for x in xs:
                car.all_reduce(x)
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=s):
                for x in xs:
                    car.all_reduce(x)
        graph_ok = True
        for rep in range(2):
            for i, x in enumerate(xs):
                x.copy_(_inp(rank, 100 + 10 * rep + i, x.numel(), torch.bfloat16))
            gr.replay()
            torch.cuda.synchronize()
            for i, x in enumerate(xs):
                graph_ok &= torch.equal(x.cpu(), _expect(100 + 10 * rep + i, x.numel(), torch.bfloat16))
        res["graph_ok"] = graph_ok
        # latency of a decode-sized message (same-GPU peers: kernel + flag overhead only)
        x = torch.randn(8192 * 8, device="cuda").to(torch.bfloat16)
        for _ in range(20):
            car.all_reduce(x)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(200):
            car.all_reduce(x)
        e1.record()
        torch.cuda.synchronize()
        res["us_per_call_128KiB"] = e0.elapsed_time(e1) * 1e3 / 200
        res["error"] = car.error()
    except Exception as e:  # noqa: BLE001
        res["exc"] = repr(e)
    q.put(res)
    dist.destroy_process_group()


def test_custom_all_reduce_two_ranks_one_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    results = [q.get(timeout=150) for _ in range(WORLD)]
    for p in procs:
        p.join(timeout=60)
    print(results)
    for r in results:
        assert "exc" not in r, r
        assert r["self_test"], r
        assert r["bad"] == [], r
        assert r["fused_bad"] == [], r
        assert r["graph_ok"], r
        assert r["error"] == 0, r
