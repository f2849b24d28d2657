"""Filter design on the host (numpy): the taps are computed once per operator and uploaded.

``firwin`` reproduces the window-method low-pass design (Hamming window, unity DC gain) the
reference gets from cusignal.firwin (sdr-holoscan/operators.py:233-236); ``decimator``
reproduces the filter length, zero pre-padding and output trimming of
``resample_poly(x, 1, down, window="hamming")`` (operators.py:300-303) so the GPU decimator
(``ops.resample_pcm``) returns exactly the samples the reference would.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


def hamming(n: int) -> np.ndarray:
    if n == 1:
        return np.ones(1)
    k = np.arange(n)
    return 0.54 - 0.46 * np.cos(2.0 * np.pi * k / (n - 1))


def firwin(numtaps: int, cutoff: float, fs: float = 2.0) -> np.ndarray:
    """Linear-phase low-pass FIR, cutoff in the units of ``fs`` (default: Nyquist = 1)."""
    fc = cutoff / (fs / 2.0)
    if not 0.0 < fc < 1.0:
        raise ValueError("cutoff must lie strictly between 0 and Nyquist")
    m = np.arange(numtaps) - (numtaps - 1) / 2.0
    h = fc * np.sinc(fc * m) * hamming(numtaps)
    return h / h.sum()


def reduce_fraction(numerator: float, denominator: float, max_up: int = 1):
    """The reference's (up, down) choice for fs_in -> fs_out (operators.py:60-66): up is
    fixed at ``max_up`` and down rounded, so 1 MS/s -> 16 kHz decimates by round(62.5) = 62
    (an effective 16.129 kHz, kept for parity)."""
    max_freq = numerator * float(max_up)
    if max_freq > 10_000_000:
        raise ValueError(f"max_freq {max_freq} is too high")
    return max_up, round(max_freq / denominator)


@dataclass
class Decimator:
    taps: np.ndarray      # zero pre-padded FIR
    down: int
    pre: int              # outputs skipped at the front (filter delay compensation)

    def n_out(self, n_in: int) -> int:
        return n_in // self.down + bool(n_in % self.down)


def decimator(down: int, up: int = 1) -> Decimator:
    if up != 1:
        raise NotImplementedError("only integer decimation (up = 1) is used by the SDR chain")
    max_rate = max(up, down)
    half_len = 10 * max_rate
    h = firwin(2 * half_len + 1, 1.0 / max_rate) * up
    n_pre_pad = down - half_len % down
    pre = (half_len + n_pre_pad) // down
    return Decimator(np.concatenate([np.zeros(n_pre_pad), h]).astype(np.float32), down, pre)
