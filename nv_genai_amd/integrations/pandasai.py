"""PandasAI LLM adapter (reference integrations/pandasai/llms/nv_aiplay.py:30-105).

``NVIDIA`` is a PandasAI ``LLM`` backed by this framework's ``ChatNVIDIA`` drop-in: the same
tunables (``model``, ``temperature``, ``max_tokens``, ``top_p``; defaults 0.1 / 1000 / 1), the
same ``type`` string, and ``call(instruction, context)`` sends ``instruction.to_string()`` as
one user turn. The endpoint is the config's ``llm.server_url`` (OpenAI/NIM protocol, e.g. this
framework's model server) or, with ``engine=``, an in-process :class:`LLMEngine` (or the
:class:`EngineService` over one). PandasAI is
optional: with it installed the class subclasses ``pandasai.llm.base.LLM``; without it the
class keeps the same duck-typed surface (the structured-data chain of this framework drives its
own LLM and does not need PandasAI).
"""
from __future__ import annotations

import logging
from typing import Any, Dict, Optional

logger = logging.getLogger(__name__)

try:  # pragma: no cover - pandasai is not part of this image
    from pandasai.llm.base import LLM as _Base
except Exception:  # noqa: BLE001
    _Base = object


class NVIDIA(_Base):
    temperature: Optional[float] = 0.1
    max_tokens: Optional[int] = 1000
    top_p: Optional[float] = 1
    model: Optional[str] = "meta/llama3-8b-instruct"

    _VALID = ("model", "temperature", "max_tokens", "top_p")

    def __init__(self, engine=None, base_url: Optional[str] = None, **kwargs: Any):
        from ..connectors.compat import ChatNVIDIA

        if engine is not None and not hasattr(engine, "engine"):   # a bare LLMEngine: serve it
            from ..serving.engine_service import EngineService

            engine = EngineService(engine)
        for k, v in kwargs.items():
            if k in self._VALID:
                setattr(self, k, v)
        if engine is None and base_url is None:
            try:
                from ..chain_server.utils import get_config

                url = get_config().llm.server_url
            except Exception:  # noqa: BLE001 - no chain-server config in this process
                url = ""
            if url:
                base_url = url if url.startswith("http") else f"http://{url}/v1"
        logger.info("PandasAI LLM %s via %s", self.model, "in-process engine" if engine else base_url or "default endpoint")
        self._chat_model = ChatNVIDIA(**self._default_params, base_url=base_url, engine=engine)
        self._prompt = ""

    @property
    def _default_params(self) -> Dict[str, Any]:
        return {"model": self.model, "temperature": self.temperature, "top_p": self.top_p,
                "max_tokens": self.max_tokens}

    @property
    def type(self) -> str:
        return "nvidia-foundational-llm"

    def call(self, instruction, context=None) -> str:
        self._prompt = instruction.to_string() if hasattr(instruction, "to_string") else str(instruction)
        return self._chat_model.invoke(self._prompt).content
