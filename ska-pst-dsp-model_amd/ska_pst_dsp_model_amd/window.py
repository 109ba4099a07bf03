"""PFBWindow — taper factories of the synthesis (matlab/PFBWindow.m:1-115).

``PFBWindow().lookup[name](input_fft_length, input_overlap)`` returns a taper
object, as the Matlab factory returns a function handle (PFBWindow.m:10-16).  The
GPU synthesis does not call the object: it reads its ``kind``/``coeffs`` and applies
the window inside the block kernel (window staged per time sample; the ``hann``
quirk becomes a per-channel gain, see ``Taper.channel_gain``).  Calling the object
on a NumPy array applies the same window on the host for callers that use the
handle directly, exactly like the Matlab handle.
"""
from __future__ import annotations

import numpy as np

from . import _lib

__all__ = ["PFBWindow", "Taper", "identity_taper", "hann"]


def hann(L: int) -> np.ndarray:
    """Matlab ``hann(L)``: symmetric, 0.5 (1 - cos(2 pi n / (L - 1)))."""
    if L == 1:
        return np.ones(1)
    n = np.arange(L)
    return 0.5 * (1.0 - np.cos(2.0 * np.pi * n / (L - 1)))


class Taper:
    """A temporal/spectral taper handle (kind + parameters)."""

    def __init__(self, kind: int, input_fft_length: int = 0, input_discard: int = 0,
                 coeffs=None, name: str = ""):
        self.kind = kind
        self.input_fft_length = int(input_fft_length)
        self.input_discard = int(input_discard)
        self.coeffs = None if coeffs is None else np.asarray(coeffs, dtype=np.float64)
        self.name = name

    # --- coefficients used by the GPU plan
    def time_window(self, nf: int) -> np.ndarray:
        """Per-time-sample window of length Nf (tukey / top_hat / custom / ones)."""
        w = np.ones(nf)
        ov = self.input_discard
        if self.kind == _lib.PFB_WINDOW_TUKEY:  # PFBWindow.m:30-34
            h = hann(2 * ov)
            w[:ov] = h[:ov]
            w[nf - ov:] = h[ov:]
        elif self.kind == _lib.PFB_WINDOW_TOP_HAT:  # PFBWindow.m:63-68
            w[:ov] = 0.0
            w[nf - ov:] = 0.0
        elif self.kind == _lib.PFB_WINDOW_CUSTOM:
            w = np.asarray(self.coeffs, dtype=np.float64)
        return w

    def channel_gain(self, n_rows: int) -> np.ndarray:
        """PFBWindow.m:72-99 quirk: ``hann`` multiplies along dim 1 (the rows).

        With rows = channels the taper is a per-channel gain:
        circshift(hann(n_rows), n_rows/2) if n_rows != Nf, else hann(Nf)."""
        if self.kind != _lib.PFB_WINDOW_HANN:
            return np.ones(n_rows)
        if n_rows != self.input_fft_length:
            return np.roll(hann(n_rows), n_rows // 2)
        return hann(self.input_fft_length)

    # --- Matlab handle semantics on the host: windowed = taper(in_dat, Nf, Ov)
    def __call__(self, in_dat, input_fft_length=None, input_discard=None):
        a = np.asarray(in_dat)
        if self.kind == _lib.PFB_WINDOW_NONE:
            return a
        if self.kind == _lib.PFB_WINDOW_HANN:
            return self.channel_gain(a.shape[0])[:, None] * a
        return a * self.time_window(a.shape[1])[None, :]

    def __repr__(self):
        return f"Taper({self.name or self.kind}, Nf={self.input_fft_length}, Ov={self.input_discard})"


def identity_taper(input=None, fft_length=None, overlap=None):
    """identity_taper.m:1-2 — the default spectral taper."""
    return input


identity_taper.kind = _lib.PFB_WINDOW_NONE  # type: ignore[attr-defined]


class PFBWindow:
    """PFBWindow.m:1-115.  ``lookup`` maps names to factories (PFBWindow.m:10-16)."""

    def __init__(self):
        self.lookup = {
            "no_window": self.no_window_factory,
            "tukey": self.tukey_factory,
            "hann": self.hann_factory,
            "top_hat": self.top_hat_factory,
        }

    def no_window_factory(self, *args):
        return Taper(_lib.PFB_WINDOW_NONE, name="no_window")

    def tukey_factory(self, input_fft_length, input_discard):
        return Taper(_lib.PFB_WINDOW_TUKEY, input_fft_length, input_discard, name="tukey")

    def top_hat_factory(self, input_fft_length, input_discard, *args):
        return Taper(_lib.PFB_WINDOW_TOP_HAT, input_fft_length, input_discard, name="top_hat")

    def hann_factory(self, input_fft_length, *args):
        return Taper(_lib.PFB_WINDOW_HANN, input_fft_length, 0, name="hann")

    def custom(self, coeffs):
        """Explicit per-sample window (not in the reference's lookup; API extension)."""
        return Taper(_lib.PFB_WINDOW_CUSTOM, len(coeffs), 0, coeffs=coeffs, name="custom")
