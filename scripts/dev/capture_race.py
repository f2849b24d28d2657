"""Does GPU work from another thread break a stream capture on this HIP runtime?
Thread A captures a graph of many matmuls on a pool stream; thread B launches matmuls at the
same time on (mode 'legacy') its default stream or (mode 'own') a pool stream of its own.
Prints whether the capture and thread B's work succeeded."""
import sys
import threading
import time

import torch

mode, cap_mode = sys.argv[1], sys.argv[2]
if len(sys.argv) > 3 and sys.argv[3] == "tuned":
    sys.path.insert(0, ".")
    from nv_genai_amd.ops.gemm_tuning import use_tuned_gemms

    print("tuned table", use_tuned_gemms())
dev = torch.device("cuda")
a = torch.randn(1024, 1024, device=dev, dtype=torch.bfloat16)
xq = torch.randn(512, 4096, device=dev, dtype=torch.bfloat16)
wq = torch.randn(6144, 4096, device=dev, dtype=torch.bfloat16)
xe = torch.randn(17, 1024, device=dev, dtype=torch.bfloat16)
we = torch.randn(4096, 1024, device=dev, dtype=torch.bfloat16)
be = torch.randn(4096, device=dev, dtype=torch.bfloat16)
torch.cuda.synchronize()
res = {}


def capture():
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    try:
        with torch.cuda.stream(s):
            x = a @ a
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s, capture_error_mode=cap_mode):
                x = a
                for _ in range(400):
                    x = x @ a
                    y = xq @ wq.t()
                    time.sleep(0.0005)
        g.replay()
        torch.cuda.synchronize()
        res["capture"] = "ok"
    except Exception as e:  # noqa: BLE001
        res["capture"] = repr(e)[:200]


def other():
    try:
        if mode == "own":
            torch.cuda.set_stream(torch.cuda.Stream())
        for i in range(200):
            y = a @ a
            z = torch.nn.functional.linear(xe[: 1 + i % 17], we, be)
            time.sleep(0.001)
        torch.cuda.current_stream().synchronize()
        res["other"] = "ok"
    except Exception as e:  # noqa: BLE001
        res["other"] = repr(e)[:200]


t1 = threading.Thread(target=capture)
t2 = threading.Thread(target=other)
t1.start()
time.sleep(0.02)
t2.start()
t1.join()
t2.join()
print(mode, cap_mode, res, flush=True)
