"""Vision-language client (Neva-22B "is it a graph?", DePlot chart->table,
examples/multimodal_rag/llm/llm_client.py:37-42). The framework serves such a model itself
(models/vision.py behind ``model_server --vlm``); this client talks to it, or to any other
OpenAI-compatible vision endpoint.

Images go as ``HumanMessage`` content with an ``image_url`` base64 JPEG data URI to any
OpenAI-compatible vision endpoint (``VLM_SERVER_URL`` / ``APP_VLM_SERVERURL``), with the Neva
steer labels (creativity / quality / complexity / verbosity) in the text. Without a configured
endpoint :class:`ImageHeuristics` answers locally from the image bytes alone (format, size,
a colour-histogram "chart-likeness" guess), so ingestion still produces searchable text.
"""
from __future__ import annotations

import base64
import os
import struct
from typing import Optional

import requests


def image_size(data: bytes):
    """(format, width, height) for PNG / JPEG / GIF bytes, else (fmt, 0, 0)."""
    if data[:8] == b"\x89PNG\r\n\x1a\n" and len(data) >= 24:
        w, h = struct.unpack(">II", data[16:24])
        return "png", w, h
    if data[:2] == b"\xff\xd8":
        i = 2
        while i + 9 < len(data):
            if data[i] != 0xFF:
                i += 1
                continue
            marker = data[i + 1]
            if marker in (0xC0, 0xC1, 0xC2):
                h, w = struct.unpack(">HH", data[i + 5:i + 9])
                return "jpeg", w, h
            seg = struct.unpack(">H", data[i + 2:i + 4])[0]
            i += 2 + seg
        return "jpeg", 0, 0
    if data[:6] in (b"GIF87a", b"GIF89a"):
        w, h = struct.unpack("<HH", data[6:10])
        return "gif", w, h
    return "unknown", 0, 0


def as_web_image(data: bytes, quality: int = 20):
    """(bytes, "png" | "jpeg") a vision endpoint can take: PNG and JPEG pass through, any other
    format PIL decodes (GIF, BMP, TIFF, WebP, ...) is re-encoded as JPEG at ``quality`` (the
    reference sends JPEG q=20: multimodal_rag/vectorstore/custom_pdf_parser.py:29-34). Bytes
    that are no image raise ValueError instead of going out mislabelled."""
    fmt, _, _ = image_size(data)
    if fmt in ("png", "jpeg"):
        return data, fmt
    import io

    from PIL import Image, UnidentifiedImageError

    try:
        im = Image.open(io.BytesIO(data))
        im.load()
    except (UnidentifiedImageError, OSError) as e:
        raise ValueError(f"not a decodable image ({len(data)} bytes)") from e
    buf = io.BytesIO()
    im.convert("RGB").save(buf, format="JPEG", quality=quality)
    return buf.getvalue(), "jpeg"


class VisionClient:
    def __init__(self, base_url: str, model: str = "ai-neva-22b", timeout: float = 120.0):
        from .http import _base

        self.base = _base(base_url)
        self.model = model
        self.timeout = timeout

    def describe(self, image: bytes, prompt: str = "Describe this image in detail",
                 max_tokens: int = 1024, **steer) -> str:
        image, fmt = as_web_image(image)
        b64 = base64.b64encode(image).decode()
        labels = ",".join(f"{k}:{v}" for k, v in steer.items())
        text = prompt + (f" [labels: {labels}]" if labels else "")
        body = {"model": self.model, "max_tokens": max_tokens, "messages": [{"role": "user", "content": [
            {"type": "text", "text": text},
            {"type": "image_url", "image_url": {"url": f"data:image/{fmt};base64,{b64}"}}]}]}
        r = requests.post(f"{self.base}/chat/completions", json=body, timeout=self.timeout)
        r.raise_for_status()
        return r.json()["choices"][0]["message"]["content"]


class ImageHeuristics:
    """Endpoint-free fallback."""

    model = "local-image-heuristics"

    def describe(self, image: bytes, prompt: str = "", max_tokens: int = 0, **steer) -> str:
        fmt, w, h = image_size(image)
        return f"An embedded {fmt} image of {w}x{h} pixels ({len(image)} bytes)."


_LOCAL = {}


class LocalDePlot:
    """In-process DePlot behind the ``describe`` contract (requests are dynamically batched)."""

    def __init__(self, deplot):
        from ..models.pix2struct import DePlotBatcher

        self.model = "google/deplot"
        self.batcher = DePlotBatcher(deplot)

    def describe(self, image: bytes, prompt: str = "", max_tokens: int = 512, **steer) -> str:
        return self.batcher.describe(image, prompt or None, min(int(max_tokens), 512))


def register_local_vision(model: str, describer) -> None:
    """Serve ``model`` in-process: ``describer`` has ``describe(image, prompt, max_tokens,
    **steer)`` — a :class:`~nv_genai_amd.models.vision.VisionLanguageModel`, a
    :class:`LocalDePlot`, or anything with that method."""
    _LOCAL[model] = describer


def load_local_vision(spec: str, device: Optional[str] = None) -> None:
    """``spec`` = "ai-neva-22b=neva-22b,ai-google-deplot=deplot" (model name = preset): load
    each preset in this process and register it (``APP_VISION_LOCAL`` at chain-server start)."""
    for item in filter(None, (x.strip() for x in spec.split(","))):
        name, preset = item.split("=", 1)
        if preset in ("deplot",) or preset.startswith("pix2struct"):
            from ..models.pix2struct import DePlot

            register_local_vision(name, LocalDePlot(DePlot(preset, device=device)))
        else:
            from ..models.vision import VisionLanguageModel

            register_local_vision(name, VisionLanguageModel(preset, device=device))


def get_vision_client(model: str = "ai-neva-22b"):
    """In-process model if one is registered under ``model``, else the configured endpoint,
    else the endpoint-free heuristics."""
    if not _LOCAL and os.environ.get("APP_VISION_LOCAL"):
        load_local_vision(os.environ["APP_VISION_LOCAL"])
    if model in _LOCAL:
        return _LOCAL[model]
    url = os.environ.get("VLM_SERVER_URL") or os.environ.get("APP_VLM_SERVERURL")
    return VisionClient(url, model) if url else ImageHeuristics()
