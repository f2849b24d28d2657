"""PandasAI adapter (integrations/pandasai.py; reference integrations/pandasai/llms/nv_aiplay.py)."""
from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine
from nv_genai_amd.integrations.pandasai import NVIDIA


class _Prompt:
    def __init__(self, text):
        self.text = text

    def to_string(self):
        return self.text


def test_pandasai_adapter_params_type_and_call_in_process():
    eng = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=4, max_batched_tokens=256, max_model_len=512,
                                 kv_cache_blocks=64), device="cpu")
    llm = NVIDIA(engine=eng, temperature=0.0, max_tokens=5, bogus=1)
    assert llm.type == "nvidia-foundational-llm"
    assert llm._default_params == {"model": "meta/llama3-8b-instruct", "temperature": 0.0, "top_p": 1,
                                   "max_tokens": 5}
    assert not hasattr(llm, "bogus")
    out = llm.call(_Prompt("df.head() of the sales table"))
    assert isinstance(out, str)
    assert llm._prompt == "df.head() of the sales table"
    assert llm.call("plain string prompt") == llm.call("plain string prompt")   # greedy: deterministic
