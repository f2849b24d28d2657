"""Cost of the first launches of the GEMV / skinny kernels in a fresh process."""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402

from nv_genai_amd import ops  # noqa: E402

x = torch.randn(1, 4096, device="cuda", dtype=torch.bfloat16)
w = torch.randn(8192, 4096, device="cuda", dtype=torch.bfloat16)
torch.cuda.synchronize()
for name, fn in (("gemv epi1", lambda: ops.gemv(x, w, 1)), ("gemv epi1 again", lambda: ops.gemv(x, w, 1)),
                 ("gemv epi0", lambda: ops.gemv(x, w, 0)), ("gemv epi2", lambda: ops.gemv(x, w, 2)),
                 ("skinny cfg1", lambda: ops.skinny_gemm(x, w, 1, 1, 0)), ("skinny cfg1 again", lambda: ops.skinny_gemm(x, w, 1, 1, 0))):
    t = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    print(f"{name}: {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
