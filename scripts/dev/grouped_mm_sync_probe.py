"""Does torch._grouped_mm synchronise with the host on ROCm (it would stall the engine's
CPU/GPU pipelining), and can it be captured in a graph?"""
import torch

dev = "cuda"
E, H, F, rows = 8, 4096, 14336, 3072
offs = torch.tensor([384 * (i + 1) for i in range(E)], dtype=torch.int32, device=dev)
a = torch.randn(rows, H, device=dev, dtype=torch.bfloat16)
wt = (torch.randn(E, 2 * F, H, device=dev, dtype=torch.bfloat16) * 0.02).transpose(1, 2)
torch._grouped_mm(a, wt, offs=offs)
torch.cuda.synchronize()
torch.cuda.set_sync_debug_mode("error")
try:
    torch._grouped_mm(a, wt, offs=offs)
    print("no host sync")
except RuntimeError as e:
    print("host sync:", str(e)[:200])
torch.cuda.set_sync_debug_mode(0)
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
try:
    with torch.cuda.stream(s):
        with torch.cuda.graph(g):
            out = torch._grouped_mm(a, wt, offs=offs)
    g.replay()
    torch.cuda.synchronize()
    ref = torch._grouped_mm(a, wt, offs=offs)
    print("graph capture ok, equal:", bool(torch.equal(out, ref)))
except Exception as e:  # noqa: BLE001
    print("graph capture failed:", repr(e)[:300])
