"""REST client of the chain server used by the playground UI, the evaluation tool and the
notebooks (RetrievalAugmentedGeneration/frontend/frontend/chat_client.py).

Every call carries the W3C ``traceparent`` of the caller's current span ("carrier"), so the
chain server's spans join the frontend's trace. ``predict`` parses the SSE stream exactly like
the reference (``json.loads(line[6:])`` of each non-empty line) and yields content chunks.
"""
from __future__ import annotations

import json
import logging
import mimetypes
import os
from typing import Dict, Generator, List, Optional, Union

import requests

from ..observability.tracing import get_tracer, inject_context

log = logging.getLogger(__name__)
tracer = get_tracer("frontend")


class ChatClient:
    def __init__(self, server_url: str, model_name: str = "meta/llama3-8b-instruct", timeout: float = 600.0):
        self.server_url = server_url.rstrip("/")
        if not self.server_url.startswith("http"):
            self.server_url = "http://" + self.server_url
        self._model_name = model_name
        self.timeout = timeout

    @property
    def model_name(self) -> str:
        return self._model_name

    def search(self, prompt: str, top_k: int = 4) -> List[Dict[str, Union[str, float]]]:
        with tracer.span("search"):
            headers = {**inject_context(), "accept": "application/json", "Content-Type": "application/json"}
            try:
                r = requests.post(f"{self.server_url}/search", headers=headers,
                                  json={"query": prompt, "top_k": top_k}, timeout=30)
                r.raise_for_status()
                return r.json().get("chunks", [])
            except Exception as e:  # noqa: BLE001
                log.error("Failed to get response from /search endpoint of chain-server: %s", e)
                return []

    def predict(self, query: str, use_knowledge_base: bool, num_tokens: int = 1024,
                temperature: float = 0.2, top_p: float = 0.7,
                history: Optional[List[dict]] = None) -> Generator[str, None, None]:
        data = {"messages": (history or []) + [{"role": "user", "content": query}],
                "use_knowledge_base": use_knowledge_base, "max_tokens": num_tokens,
                "temperature": temperature, "top_p": top_p}
        with tracer.span("predict", {"use_knowledge_base": use_knowledge_base}) as span:
            try:
                with requests.post(f"{self.server_url}/generate", stream=True, json=data, timeout=self.timeout,
                                   headers=inject_context()) as r:
                    r.raise_for_status()
                    out = []
                    for line in r.iter_lines():
                        raw = line.decode("UTF-8")
                        if not raw:
                            continue
                        try:
                            choices = json.loads(raw[6:]).get("choices", [])
                        except Exception as e:
                            raise ValueError(f"Invalid response json: {raw}") from e
                        chunk = choices[0].get("message", {}).get("content", "") if choices else ""
                        out.append(chunk)
                        yield chunk
                    if span is not None:
                        span.set_attribute("response", "".join(out)[:4000])
            except Exception as e:  # noqa: BLE001
                log.error("Failed to get response from /generate endpoint of chain-server: %s", e)
                yield ("Failed to get response from /generate endpoint of chain-server. Check if the fastapi "
                       "server in chain-server is up. Refer to chain-server logs for details.")

    def upload_documents(self, file_paths: List[str]) -> None:
        with tracer.span("upload_documents"):
            for fpath in file_paths:
                mime, _ = mimetypes.guess_type(fpath)
                with open(fpath, "rb") as fh:
                    r = requests.post(f"{self.server_url}/documents", headers={**inject_context(), "accept": "application/json"},
                                      files={"file": (os.path.basename(fpath), fh, mime or "application/octet-stream")},
                                      timeout=self.timeout)
                if r.status_code == 500:
                    raise ValueError(r.json().get("message", "Failed to upload document"))

    def delete_documents(self, file_name: str) -> str:
        with tracer.span("delete_documents"):
            r = requests.delete(f"{self.server_url}/documents", params={"filename": file_name},
                                headers={**inject_context(), "accept": "application/json"}, timeout=30)
            r.raise_for_status()
            return r.json().get("message", "")

    def get_uploaded_documents(self) -> List[str]:
        with tracer.span("get_documents"):
            r = requests.get(f"{self.server_url}/documents", headers={**inject_context(), "accept": "application/json"},
                             timeout=30)
            r.raise_for_status()
            return r.json().get("documents", [])
