"""WAV → FM-modulated complex baseband → UDP packets (SURVEY.md §2.A E2 file-replay;
experimental/fm-asr-streaming-rag/file-replay/wav_replay.py:83-214).

FM modulation: resample the audio to the I/Q rate, integrate, phase = 2π·Δf·∫audio,
samples = e^{j·phase} (complex64). Packets carry an 8-byte little-endian counter followed by
``packet_size`` bytes of I/Q, paced in real time (or as fast as possible with ``realtime=False``).

``python -m nv_genai_amd.dsp.replay --file talk.wav --dst-port 5005``
"""
from __future__ import annotations

import argparse
import socket
import struct
import time
import wave
from typing import Iterator, Optional

import numpy as np


def read_wav(path: str) -> tuple:
    """-> (mono float32 in [-1, 1], sample rate). PCM16/PCM32/float32 WAV."""
    with wave.open(path, "rb") as w:
        fs, ch, sw, n = w.getframerate(), w.getnchannels(), w.getsampwidth(), w.getnframes()
        raw = w.readframes(n)
    if sw == 2:
        a = np.frombuffer(raw, dtype="<i2").astype(np.float32) / 32768.0
    elif sw == 4:
        a = np.frombuffer(raw, dtype="<i4").astype(np.float32) / 2147483648.0
    elif sw == 1:
        a = (np.frombuffer(raw, dtype=np.uint8).astype(np.float32) - 128.0) / 128.0
    else:
        raise ValueError(f"unsupported sample width {sw}")
    if ch > 1:
        a = a.reshape(-1, ch).mean(axis=1)
    return a, fs


def write_wav(path: str, pcm16: np.ndarray, fs: int) -> None:
    with wave.open(path, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(int(fs))
        w.writeframes(np.asarray(pcm16, dtype="<i2").tobytes())


def fm_modulate(audio: np.ndarray, fs_in: float, fs_out: float, deviation: float = 100_000.0,
                phase0: float = 0.0) -> tuple:
    """-> (complex64 I/Q at fs_out, final phase for the next chunk)."""
    n = int(len(audio) * fs_out / fs_in)
    # band-limited resampling through the FFT (as scipy.signal.resample)
    spec = np.fft.rfft(audio.astype(np.float64))
    m = n // 2 + 1
    out = np.zeros(m, dtype=np.complex128)
    k = min(m, spec.shape[0])
    out[:k] = spec[:k]
    if n % 2 == 0 and k == m and len(audio) > n:
        out[-1] = out[-1].real
    up = np.fft.irfft(out, n) * (n / max(1, len(audio)))
    phase = phase0 + 2.0 * np.pi * deviation * np.cumsum(up) / fs_out
    return np.exp(1j * phase).astype(np.complex64), float(phase[-1] if len(phase) else phase0)


def packets(iq: np.ndarray, packet_size: int = 1472, counter0: int = 0) -> Iterator[bytes]:
    data = iq.tobytes()
    c = counter0
    for i in range(0, len(data), packet_size):
        yield struct.pack("<Q", c) + data[i:i + packet_size]
        c += 1


def replay(path: str, dst_ip: str = "127.0.0.1", dst_port: int = 5005, fs_out: float = 1e6,
           packet_size: int = 1472, chunk_time: float = 2.0, total_time: float = 0.0,
           realtime: bool = True, sock: Optional[socket.socket] = None) -> int:
    """Stream the file (looping until ``total_time`` if set); returns packets sent."""
    audio, fs = read_wav(path)
    s = sock or socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    total_time = total_time or len(audio) / fs
    hop = int(chunk_time * fs)
    sent, elapsed, phase, counter = 0, 0.0, 0.0, 0
    while elapsed < total_time:
        for i in range(0, len(audio), hop):
            chunk = audio[i:i + hop]
            iq, phase = fm_modulate(chunk, fs, fs_out, phase0=phase)
            pk = list(packets(iq, packet_size, counter))
            counter += len(pk)
            dt = (len(chunk) / fs) / max(1, len(pk))
            for p in pk:
                s.sendto(p, (dst_ip, dst_port))
                sent += 1
                if realtime:
                    time.sleep(dt)
            elapsed += len(chunk) / fs
            if elapsed >= total_time:
                break
    return sent


def main(argv=None):
    ap = argparse.ArgumentParser(description="Replay a WAV file as FM-modulated I/Q UDP packets")
    ap.add_argument("--file", required=True)
    ap.add_argument("--dst-ip", default="127.0.0.1")
    ap.add_argument("--dst-port", type=int, default=5005)
    ap.add_argument("--sample-rate", type=float, default=1e6)
    ap.add_argument("--packet-size", type=int, default=1472)
    ap.add_argument("--total-time", type=float, default=0.0)
    ap.add_argument("--fast", action="store_true", help="do not pace packets in real time")
    a = ap.parse_args(argv)
    n = replay(a.file, a.dst_ip, a.dst_port, a.sample_rate, a.packet_size, total_time=a.total_time,
               realtime=not a.fast)
    print(f"sent {n} packets")


if __name__ == "__main__":
    main()
