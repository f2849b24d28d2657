"""Eight ranks on one GPU: the custom all-reduce kernels in an engine-like sequence (a large
GEMM, then one-shot, two-shot, fused add+RMSNorm and the logits all-gather), eagerly and from
a captured hipGraph, to see whether every call meets its peers (sticky timeout code 0) and the
sums are exact. Usage: python ar8_probe.py [--world 8] [--blocks N] [--iters 50] [--graph].
Prints one JSON line per rank (rank 0 last)."""
import argparse
import json
import os
import socket
import sys
import time

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, args, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(args.world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    if args.queues:
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.queues)
    if args.blocks:
        os.environ["NGA_CUSTOM_AR_BLOCKS"] = str(args.blocks)
    import torch.distributed as dist

    from nv_genai_amd.parallel.custom_ar import CustomAllReduce

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=args.world)
    res = {"rank": rank}
    try:
        car = CustomAllReduce(None, capacity_mb=16, timeout_s=args.timeout)
        res["self_test"], res["max_blocks"], res["ranks_per_device"] = car.enabled, car.max_blocks, car.ranks_per_device
        dev = torch.device("cuda", 0)
        g = torch.Generator().manual_seed(rank)
        a = torch.randn(2048, 2048, generator=g).to(dev, torch.bfloat16)
        small = torch.full((4, 2048), float(rank + 1), device=dev, dtype=torch.bfloat16)
        big = torch.full((512, 2048), float(rank + 1), device=dev, dtype=torch.bfloat16)
        resid = torch.zeros(4, 2048, device=dev, dtype=torch.bfloat16)
        w = torch.ones(2048, device=dev, dtype=torch.bfloat16)
        shard = torch.full((4, 4096), float(rank), device=dev)
        o_small, o_big = torch.empty_like(small), torch.empty_like(big)
        o_norm = torch.empty_like(small)
        o_gather = torch.empty(4, 4096 * args.world, device=dev)

        def seq():
            for _ in range(args.gemms):
                torch.matmul(a, a)
            car.all_reduce(small, out=o_small)
            car.all_reduce(big, out=o_big)
            car.all_reduce_add_rmsnorm(small, resid, w, 1e-5, out=o_norm)
            car.all_gather(shard, out=o_gather)

        tot = args.world * (args.world + 1) / 2
        bad = 0
        graph = None
        if args.graph:
            seq()
            torch.cuda.synchronize()
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph, stream=s):
                    seq()
            torch.cuda.synchronize()
        dist.barrier()
        t0 = time.time()
        for it in range(args.iters):
            graph.replay() if graph is not None else seq()
            if it % 10 == 9 or it == args.iters - 1:
                torch.cuda.synchronize()
                bad += int(not (torch.all(o_small == tot) and torch.all(o_big == tot)))
                want = torch.arange(args.world, device=dev).float().repeat_interleave(4096)
                bad += int(not torch.equal(o_gather[0], want))
        torch.cuda.synchronize()
        res["s_per_iter"] = round((time.time() - t0) / args.iters, 5)
        res["bad_checks"] = bad
        res["error"] = car.error()
        res["algo_counts"] = dict(car.algo_counts)
    except Exception as e:  # noqa: BLE001
        res["exc"] = repr(e)[:500]
    q.put(res)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--blocks", type=int, default=0)
    ap.add_argument("--queues", type=int, default=0)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--gemms", type=int, default=4)
    ap.add_argument("--timeout", type=float, default=2.0)
    ap.add_argument("--graph", action="store_true")
    args = ap.parse_args()
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, args, port, q)) for r in range(args.world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in ps], key=lambda r: -r["rank"])
    for p in ps:
        p.join(60)
    summary = {"args": vars(args), "ok": all("exc" not in r and r["error"] == 0 and r["bad_checks"] == 0 for r in res),
               "errors": [r.get("error") for r in res], "bad": [r.get("bad_checks") for r in res],
               "s_per_iter": max(r.get("s_per_iter", 0) for r in res), "r0": res[-1]}
    print(json.dumps(summary), flush=True)


if __name__ == "__main__":
    main()
