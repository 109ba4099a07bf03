"""Purity metrics and alignment of the reference's verification harness
(``python/verify/util.py:15-43``, ``python/verify/purity.py:76-88,165-283``), so the
``hip`` backend can be scored exactly as the reference scores its backends.

Host-side NumPy on the (small) metric arrays; the data they score comes off the device.
"""
from __future__ import annotations

import numpy as np

from .config import as_rational

__all__ = ["spurious", "total_spurious", "mean_spurious", "max_spurious", "dB",
           "purity_alignment", "impulse_purity", "tone_purity"]


def spurious(a):
    """util.py:15-18: the array with its largest element zeroed."""
    b = np.array(a, copy=True)
    b[np.argmax(b)] = 0.0
    return b


def dB(a):
    """util.py:39-43 (``a`` already in power)."""
    return 10.0 * np.log10(np.abs(np.array(a, copy=True)) + 1e-13)


def total_spurious(a):
    """util.py:21-24."""
    return dB(np.sum(spurious(np.abs(a) ** 2)))


def mean_spurious(a):
    """util.py:27-30."""
    return dB(np.mean(spurious(np.abs(a) ** 2)))


def max_spurious(a):
    """util.py:33-36."""
    return dB(np.amax(spurious(np.abs(a) ** 2)))


def purity_alignment(channels: int, os_factor, input_fft_length: int, input_overlap: int,
                     fir_filter_taps: int, blocks: int) -> dict:
    """purity.py:76-88: block size, sample counts and the shift between a test vector
    and the synthesised output (overlap discard + FIR group delay)."""
    o = as_rational(os_factor)
    block_size = input_fft_length * o.de // o.nu * channels
    output_sample_shift = input_overlap * o.de // o.nu * channels
    return {"normalize": input_fft_length * channels, "block_size": block_size,
            "fft_size": 2 * block_size, "n_samples": block_size * blocks,
            "output_sample_shift": output_sample_shift,
            "total_sample_shift": output_sample_shift + (fir_filter_taps - 1) // 2}


def impulse_purity(synth: np.ndarray, offset: int, total_sample_shift: int) -> dict:
    """Score a synthesised temporal impulse (TestImpulse.m:46-73 criteria): the output
    is aligned by ``total_sample_shift`` (purity.py:276-283) and the power outside the
    impulse sample is summarised by the util.py metrics."""
    y = np.asarray(synth).reshape(-1)
    pos = offset - total_sample_shift
    peak = int(np.argmax(np.abs(y)))
    p = np.abs(y) ** 2
    p = p / p.max()
    return {"peak_index": peak, "expected_index": pos, "total_spurious": float(total_spurious(np.sqrt(p))),
            "max_spurious": float(max_spurious(np.sqrt(p))),
            "mean_spurious": float(mean_spurious(np.sqrt(p)))}


def tone_purity(synth: np.ndarray) -> dict:
    """Score a synthesised tone (TestPureTone.m:55-89): spectrum power normalised to the
    tone bin, util.py metrics over the remaining bins."""
    y = np.asarray(synth).reshape(-1)
    spec = np.abs(np.fft.fft(y)) ** 2
    spec = spec / spec.max()
    return {"peak_bin": int(np.argmax(spec)), "total_spurious": float(total_spurious(np.sqrt(spec))),
            "max_spurious": float(max_spurious(np.sqrt(spec))),
            "mean_spurious": float(mean_spurious(np.sqrt(spec)))}
