"""Wall time of an engine's first steps (startup costs: lazy kernel loading, graph capture)."""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402

from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine, SamplingParams  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
t0 = time.perf_counter()
eng = LLMEngine(EngineConfig(model="llama3-8b", max_num_seqs=B, max_batched_tokens=32768, max_model_len=8192,
                             graph_batch_sizes=(B,), enable_prefix_caching=False, mixed_prefill_tokens=0,
                             token_alignment=1))
torch.cuda.synchronize()
print(f"engine init {time.perf_counter() - t0:.3f} s", flush=True)
reqs = [eng.add_request(list(range(100, 1450)), SamplingParams(temperature=0.7, max_tokens=8, ignore_eos=True))
        for _ in range(B)]
for i in range(6):
    t = time.perf_counter()
    eng.step()
    torch.cuda.synchronize()
    print(f"step {i}: {1e3 * (time.perf_counter() - t):.1f} ms  captures={eng.stats.get('graph_captures')}", flush=True)
