"""SDR burst pipeline and UDP I/Q receiver (sdr-holoscan/app.py:28-75,
operators.py:86-352, params.yml).

Reference flow (Holoscan operators): network_rx → pkt_format → lowpassfilt (101-tap Hamming
FIR, 100 kHz @ 1 MS/s) → demodulate (diff(unwrap(angle))) → resample (1 MS/s → ~16 kHz,
gain 10) → pcm_to_asr (int16 → ASR queue). Here each burst is three HIP kernels on one stream
(``ops.fir_c64`` / ``ops.fm_demod`` / ``ops.resample_pcm``) and a single D2H copy of the PCM.

``stateful=False`` (default) matches the reference exactly: every burst is filtered from zero
initial state and demodulated/decimated on its own (so each burst loses one demod sample and
has a filter transient at its start). ``stateful=True`` carries the FIR history, the last
sample for the demodulator and the decimator's input tail across bursts, so consecutive
bursts produce the same PCM as processing the whole stream at once.
"""
from __future__ import annotations

import logging
import socket
import threading
from queue import Queue
from typing import Optional

import numpy as np
import torch

from .. import ops
from .design import decimator, firwin, reduce_fraction

log = logging.getLogger(__name__)


class SDRPipeline:
    def __init__(self, sample_rate: float = 1_000_000, cutoff: float = 100_000, numtaps: int = 101,
                 sample_rate_out: float = 16_000, gain: float = 10.0, device: Optional[str] = None,
                 stateful: bool = False):
        self.device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        self.fs_in, self.fs_out, self.gain, self.stateful = float(sample_rate), float(sample_rate_out), gain, stateful
        self.taps = torch.tensor(firwin(numtaps, cutoff, sample_rate), dtype=torch.float32, device=self.device)
        up, down = reduce_fraction(max(self.fs_in, self.fs_out), min(self.fs_in, self.fs_out))
        self.dec = decimator(down, up)
        self.dec_taps = torch.from_numpy(self.dec.taps).to(self.device)
        self.reset()

    def reset(self):
        self.hist = torch.zeros(self.taps.numel() - 1, dtype=torch.complex64, device=self.device)
        self.prev: Optional[complex] = None
        # decimator stream state: demod samples not yet fully consumed + absolute index of tail[0]
        self.tail = torch.zeros(0, dtype=torch.float32, device=self.device)
        self.tail_start = 0
        self.n_emitted = 0
        self.n_seen = 0

    def process(self, iq: torch.Tensor):
        """complex64 burst → (float32 audio, int16 PCM) on the pipeline device."""
        x = iq.to(self.device, torch.complex64).contiguous()
        if not self.stateful:
            lp = ops.fir_c64(x, self.taps)
            dm = ops.fm_demod(lp)
            d = self.dec
            return ops.resample_pcm(dm, self.dec_taps, d.down, d.pre, d.n_out(dm.numel()), self.gain)
        lp = ops.fir_c64(x, self.taps, self.hist)
        nt = self.taps.numel() - 1
        self.hist = torch.cat([self.hist, x])[-nt:].contiguous() if nt else self.hist
        dm = ops.fm_demod(lp, self.prev)
        self.prev = complex(lp[-1].item()) if lp.numel() else self.prev
        return self._decimate_stream(dm)

    def _decimate_stream(self, dm: torch.Tensor):
        """Emit every decimated output whose input window is complete (stream alignment:
        output m of the whole stream reads samples (m + pre)·down - k)."""
        d = self.dec
        buf = torch.cat([self.tail, dm])
        self.n_seen += dm.numel()
        last = self.n_seen - 1                     # absolute index of the newest sample
        m_end = last // d.down - d.pre + 1         # outputs m with (m + pre)·down <= last
        m0 = self.n_emitted
        if m_end <= m0:
            return (torch.zeros(0, device=self.device), torch.zeros(0, dtype=torch.int16, device=self.device))
        # window start must be a multiple of `down` so the kernel's index math stays integral
        start = self.tail_start
        pre_w = m0 + d.pre - start // d.down
        yf, yi = ops.resample_pcm(buf, self.dec_taps, d.down, pre_w, m_end - m0, self.gain)
        self.n_emitted = m_end
        # keep enough history for the next outputs: from (m_end + pre)·down - (ntaps - 1)
        keep_from = max(0, (m_end + d.pre) * d.down - (self.dec_taps.numel() - 1))
        keep_from -= keep_from % d.down
        keep_from = max(keep_from, start)
        self.tail = buf[keep_from - start:].contiguous()
        self.tail_start = keep_from
        return yf, yi


def pcm_bytes(pcm: torch.Tensor) -> bytes:
    return pcm.cpu().numpy().astype("<i2").tobytes()


class UDPReceiver(threading.Thread):
    """Receives I/Q packets (8-byte counter header + complex64 payload), accumulates
    ``batch_size`` payload bytes and pushes each burst (numpy complex64) to ``out``
    (network_rx + pkt_format operators)."""

    def __init__(self, out: Queue, ip: str = "0.0.0.0", port: int = 5005, batch_size: int = 47104,
                 header_bytes: int = 8, max_payload: int = 1472):
        super().__init__(daemon=True)
        self.out, self.batch, self.hdr, self.max_payload = out, batch_size, header_bytes, max_payload
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM, socket.IPPROTO_UDP)
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 49_000_000)
        self.sock.bind((ip, port))
        self.sock.settimeout(0.2)
        self.port = self.sock.getsockname()[1]
        self._stop_ev = threading.Event()
        self.bytes = 0

    def run(self):
        buf = bytearray()
        while not self._stop_ev.is_set():
            try:
                pkt = self.sock.recv(self.hdr + self.max_payload)
            except socket.timeout:
                continue
            except OSError:
                break
            buf.extend(pkt[self.hdr:])
            self.bytes += len(pkt)
            if len(buf) >= self.batch:
                n = len(buf) // 8 * 8
                self.out.put(np.frombuffer(bytes(buf[:n]), dtype=np.complex64).copy())
                del buf[:n]
        self.sock.close()

    def stop(self):
        self._stop_ev.set()


def run_sdr(receiver_q: Queue, pipeline: SDRPipeline, pcm_q: Queue, stop: threading.Event):
    """pkt_format → DSP → pcm_to_asr loop (one thread; the GPU does the signal processing)."""
    while not stop.is_set():
        try:
            burst = receiver_q.get(timeout=0.2)
        except Exception:  # queue.Empty
            continue
        _, pcm = pipeline.process(torch.from_numpy(burst))
        pcm_q.put(pcm_bytes(pcm))
