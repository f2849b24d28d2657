"""One-rank RCCL init through the same rendezvous path as parallel/dist.py (env:// store,
per-incarnation PrefixStore, device_id): all-reduce + barrier + broadcast on the GPU."""
import datetime
import os

import torch
import torch.distributed as dist

os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29611", RANK="0", WORLD_SIZE="1")
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
td = datetime.timedelta(seconds=60)
store, _, _ = next(dist.rendezvous("env://", 0, 1, timeout=td))
store = dist.PrefixStore("nga0/", store)
dist.init_process_group(backend="nccl", store=store, rank=0, world_size=1, timeout=td, device_id=dev)
t = torch.ones(4, device=dev)
dist.all_reduce(t)
dist.barrier()
dist.broadcast(t, src=0)
torch.cuda.synchronize()
print("rccl ok", t.tolist(), dist.get_backend())
dist.destroy_process_group()
