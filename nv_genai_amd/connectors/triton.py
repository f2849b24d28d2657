"""Client for the Triton ``generate`` / ``generate_stream`` extension (SURVEY.md §2.A E9;
experimental/AzureML/trt_llm_azureml.py: ``TensorRTLLM`` LLM + ``HttpTritonClient`` with
text_input / max_tokens / top_k / top_p / temperature / length_penalty / repetition_penalty /
random_seed / beam_width / stream). Works against this framework's model server, which serves
the same extension at ``/v2/models/{model}/generate[_stream]``."""
from __future__ import annotations

import json
from typing import Iterator, Optional

import requests


class TritonLLM:
    def __init__(self, server_url: str, model_name: str = "ensemble", tokens: int = 100, temperature: float = 1.0,
                 top_k: int = 1, top_p: float = 0.0, beam_width: int = 1, repetition_penalty: float = 1.0,
                 length_penalty: float = 1.0, seed: Optional[int] = 42, timeout: float = 600.0):
        self.url = server_url.rstrip("/")
        if not self.url.startswith("http"):
            self.url = "http://" + self.url
        self.model_name = model_name
        self.defaults = dict(max_tokens=tokens, temperature=temperature, top_k=top_k, top_p=top_p,
                             beam_width=beam_width, repetition_penalty=repetition_penalty,
                             length_penalty=length_penalty, random_seed=seed)
        self.timeout = timeout

    def _body(self, prompt: str, **kw):
        b = {"text_input": prompt, **self.defaults, **{k: v for k, v in kw.items() if v is not None}}
        if b.get("top_p", 0) <= 0:
            b["top_p"] = 1.0
        return b

    def invoke(self, prompt: str, **kw) -> str:
        r = requests.post(f"{self.url}/v2/models/{self.model_name}/generate", json=self._body(prompt, **kw),
                          timeout=self.timeout)
        r.raise_for_status()
        return r.json()["text_output"]

    __call__ = invoke

    def stream(self, prompt: str, **kw) -> Iterator[str]:
        with requests.post(f"{self.url}/v2/models/{self.model_name}/generate_stream", json=self._body(prompt, **kw),
                           stream=True, timeout=self.timeout) as r:
            r.raise_for_status()
            for line in r.iter_lines(decode_unicode=True):
                if line and line.startswith("data:"):
                    yield json.loads(line[5:])["text_output"]
