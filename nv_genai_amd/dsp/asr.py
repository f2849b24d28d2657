"""Speech recognition hand-off for the FM streaming RAG (reference:
sdr-holoscan/riva_asr.py:27-146 — a thread streams PCM16 to Riva ``StreamingRecognize`` with
interim results, posts every *final* transcript to the chain server's
``/storeStreamingText`` ({"transcript", "source_id": "Channel 0", "timestamp"}) and every
final/partial transcript to the frontend (``/app/update_finalized_transcript``,
``/app/update_running_transcript``, de-duplicating repeated partials).

Riva is an external microservice with no equivalent in this image, so recognisers are
pluggable behind ``ASRBackend.stream(pcm_chunks) -> iterator of (text, is_final)``:

* ``HTTPTranscriptionASR`` — buffers ``segment_s`` seconds of PCM, wraps it as WAV and POSTs
  it to an OpenAI-compatible ``/v1/audio/transcriptions`` endpoint (any ASR server);
* ``ScriptedASR`` — replays a known transcript at the audio's pace (tests and demos).
"""
from __future__ import annotations

import datetime
import io
import logging
import threading
import wave
from queue import Empty, Queue
from typing import Iterable, Iterator, List, Optional, Tuple

import requests

log = logging.getLogger(__name__)


class ASRBackend:
    def stream(self, pcm_chunks: Iterable[bytes]) -> Iterator[Tuple[str, bool]]:
        raise NotImplementedError


def pcm_to_wav(pcm: bytes, rate: int) -> bytes:
    b = io.BytesIO()
    with wave.open(b, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(rate)
        w.writeframes(pcm)
    return b.getvalue()


class HTTPTranscriptionASR(ASRBackend):
    def __init__(self, url: str, model: str = "asr", sample_rate: int = 16000, segment_s: float = 5.0,
                 language: str = "en", timeout: float = 60.0):
        self.url = url.rstrip("/")
        self.model, self.rate, self.segment, self.lang, self.timeout = model, sample_rate, segment_s, language, timeout

    def _transcribe(self, pcm: bytes) -> str:
        files = {"file": ("segment.wav", pcm_to_wav(pcm, self.rate), "audio/wav")}
        r = requests.post(f"{self.url}/v1/audio/transcriptions", files=files,
                          data={"model": self.model, "language": self.lang}, timeout=self.timeout)
        r.raise_for_status()
        return r.json().get("text", "")

    def stream(self, pcm_chunks):
        need = int(self.segment * self.rate) * 2
        buf = bytearray()
        for c in pcm_chunks:
            buf.extend(c)
            if len(buf) >= need:
                text = self._transcribe(bytes(buf))
                buf.clear()
                if text:
                    yield text, True
        if buf:
            text = self._transcribe(bytes(buf))
            if text:
                yield text, True


class ScriptedASR(ASRBackend):
    """Emits ``words_per_second`` words of a script per second of audio: partial results every
    chunk, a final result at each sentence end."""

    def __init__(self, script: str, sample_rate: int = 16000, words_per_second: float = 2.5):
        self.words = script.split()
        self.rate, self.wps = sample_rate, words_per_second

    def stream(self, pcm_chunks):
        audio_s, emitted, sentence = 0.0, 0, []
        for c in pcm_chunks:
            audio_s += len(c) / 2 / self.rate
            target = min(len(self.words), int(audio_s * self.wps))
            while emitted < target:
                w = self.words[emitted]
                emitted += 1
                sentence.append(w)
                if w.endswith((".", "?", "!")):
                    yield " ".join(sentence), True
                    sentence = []
            if sentence:
                yield " ".join(sentence), False
        if sentence:
            yield " ".join(sentence), True


class TranscriptExporter(threading.Thread):
    """Pulls PCM from ``pcm_q``, runs the ASR backend and exports transcripts (RivaThread)."""

    def __init__(self, pcm_q: Queue, asr: ASRBackend, database_uri: Optional[str] = None,
                 frontend_uri: Optional[str] = None, source_id: str = "Channel 0", session=None):
        super().__init__(daemon=True)
        self.q, self.asr, self.db, self.fe, self.source = pcm_q, asr, database_uri, frontend_uri, source_id
        self.http = session or requests.Session()
        self._stop_ev = threading.Event()
        self._prev_partial: Optional[str] = None
        self.finals: List[str] = []

    def _chunks(self):
        while not self._stop_ev.is_set():
            try:
                yield self.q.get(timeout=0.2)
            except Empty:
                continue

    def _post(self, url: str, data: dict):
        try:
            self.http.post(url, json=data, timeout=10)
        except requests.exceptions.RequestException as e:
            log.error("failed to post to %s: %s", url, e)

    def export(self, text: str, final: bool):
        now = datetime.datetime.now().strftime("%Y-%m-%d %H:%M:%S")
        if final:
            self.finals.append(text)
            if self.db:
                self._post(f"http://{self.db}/storeStreamingText",
                           {"transcript": text, "source_id": self.source, "timestamp": now})
            if self.fe:
                self._post(f"http://{self.fe}/app/update_finalized_transcript", {"transcript": f"[{now}] {text}"})
        else:
            if text == self._prev_partial:
                return
            self._prev_partial = text
            if self.fe:
                self._post(f"http://{self.fe}/app/update_running_transcript", {"transcript": f"[{now}] {text}"})

    def run(self):
        for text, final in self.asr.stream(self._chunks()):
            self.export(text, final)
            if self._stop_ev.is_set():
                break

    def stop(self):
        self._stop_ev.set()
