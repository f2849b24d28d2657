"""Text-to-speech hand-off for the playground (reference:
RetrievalAugmentedGeneration/frontend/frontend/tts_utils.py:77-127 — Riva
``synthesize_online`` streaming int16 PCM chunks, with answers segmented for Riva's
400-character limit by inserting " . " at the last space before every 300 characters).

Riva itself is an external service; ``HTTPSpeechTTS`` targets any OpenAI-compatible
``/v1/audio/speech`` endpoint that returns WAV or raw PCM16 and yields (rate, int16 array)
chunks like the reference generator.
"""
from __future__ import annotations

import io
import wave
from typing import Iterator, Tuple

import numpy as np
import requests


def segment_for_tts(text: str, limit: int = 300) -> str:
    """The reference's segmentation, including its index drift: each inserted " . " shifts
    later positions, and the search restarts from the growing string."""
    for i in range(len(text) // limit + 1):
        idx = text.rfind(" ", 0, (i + 1) * limit)
        text = text[:idx] + " . " + text[idx:]
    return text


class HTTPSpeechTTS:
    def __init__(self, url: str, model: str = "tts", voice: str = "default", sample_rate: int = 44100,
                 chunk_samples: int = 8192, timeout: float = 60.0):
        self.url, self.model, self.voice = url.rstrip("/"), model, voice
        self.rate, self.chunk, self.timeout = sample_rate, chunk_samples, timeout

    def synthesize(self, text: str, voice: str = None) -> Iterator[Tuple[int, np.ndarray]]:
        r = requests.post(f"{self.url}/v1/audio/speech", timeout=self.timeout,
                          json={"model": self.model, "input": segment_for_tts(text), "voice": voice or self.voice,
                                "response_format": "wav"})
        r.raise_for_status()
        data, rate = r.content, self.rate
        if data[:4] == b"RIFF":
            with wave.open(io.BytesIO(data)) as w:
                rate = w.getframerate()
                data = w.readframes(w.getnframes())
        pcm = np.frombuffer(data, dtype="<i2")
        for i in range(0, len(pcm), self.chunk):
            yield rate, pcm[i:i + self.chunk]
        yield rate, np.frombuffer(b"", dtype=np.int16)
