"""Time lazy step-graph captures of a TP=2 rank's shapes in ONE process (heads 16 / kv 4, FFN and
vocab halved, hidden 4,096): each phase of _capture_step_graph for chosen (token bucket,
decode-row bucket) keys — isolates a slow warm-up from the two-process rehearsal."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ.setdefault("NGA_TRACE_CAPTURE", "1")
import torch  # noqa: E402

from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine  # noqa: E402
from nv_genai_amd.models.config import llama_config  # noqa: E402
from nv_genai_amd.parallel.dist import ParallelContext  # noqa: E402

half = llama_config("llama3-8b", heads=16, kv_heads=4, ffn=7168, vocab_size=64128, layers=int(sys.argv[1]) if len(sys.argv) > 1 else 32)
eng = LLMEngine(EngineConfig(model="llama3-8b", max_num_seqs=64, max_batched_tokens=32768, max_model_len=8192,
                             graph_batch_sizes=(1, 8, 64), mixed_prefill_tokens=4096),
                device="cuda", pctx=ParallelContext(), model_cfg=half)
for key in [(1024, 0), (3328, 64), (3328, 8), (4096, 64), (3072, 64), (3328, 32)]:
    t = time.perf_counter()
    eng._capture_step_graph(key)
    print(key, "capture", round(time.perf_counter() - t, 3), "s", flush=True)
