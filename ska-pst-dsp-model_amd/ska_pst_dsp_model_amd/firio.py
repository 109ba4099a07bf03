"""Plan-time FIR inputs: tap files and prototype filter design.

    read_fir_filter_coeff          matlab/read_fir_filter_coeff.m:11-18
    design_PFB_FIR_filter          matlab/design_PFB_FIR_filter.m:24-52
    design_PFB_FIR_filter_two_stage matlab/design_PFB_FIR_filter_two_stage.m:19-84

The Matlab designs use ``fdesign.lowpass('N,Fp,Fst', n, Fp, Fst)`` +
``design(..., 'firls', 'Wstop', 15)``; the equivalent least-squares design is
``scipy.signal.firls(n + 1, [0, Fp, Fst, 1], [1, 1, 0, 0], weight=[1, 15])`` on the
same Nyquist-normalised band edges.  Matlab is not available to confirm the taps
bit-for-bit; the designed taps are pinned as fixtures in ``tests/golden``.
"""
from __future__ import annotations

import os

import numpy as np

from .config import as_rational

__all__ = ["read_fir_filter_coeff", "design_PFB_FIR_filter", "design_PFB_FIR_filter_two_stage",
           "save_fir_filter_coeff"]


def read_fir_filter_coeff(file_path: str) -> np.ndarray:
    """.mat field ``hQ`` or ``h`` (transposed), else a raw numeric file (read_fir_filter_coeff.m)."""
    ext = os.path.splitext(file_path)[1].lower()
    if ext == ".mat":
        from scipy.io import loadmat
        m = loadmat(file_path)
        for key in ("hQ", "h"):
            if key in m:
                return np.asarray(m[key], dtype=np.float64).ravel()
        raise KeyError(f"{file_path}: no 'h' or 'hQ' field")
    if ext == ".npy":
        return np.load(file_path, allow_pickle=False).astype(np.float64).ravel()
    return np.loadtxt(file_path, dtype=np.float64).ravel()


def save_fir_filter_coeff(file_path: str, h) -> str:
    """Write taps as a .mat (field ``h``) or .npy / text file."""
    ext = os.path.splitext(file_path)[1].lower()
    h = np.asarray(h, dtype=np.float64).ravel()
    if ext == ".mat":
        from scipy.io import savemat
        savemat(file_path, {"h": h[None, :]})
    elif ext == ".npy":
        np.save(file_path, h)
    else:
        np.savetxt(file_path, h)
    return file_path


def _firls(numtaps, fp, fs, wstop=15.0):
    from scipy.signal import firls
    return firls(numtaps, [0.0, fp, fs, 1.0], [1.0, 1.0, 0.0, 0.0], weight=[1.0, wstop])


def design_PFB_FIR_filter(n_chan: int, os_factor, n_taps_per_chan: int) -> np.ndarray:
    """design_PFB_FIR_filter.m:24-52 — firls prototype of order n_chan*n_taps_per_chan."""
    os_ = as_rational(os_factor)
    OS = os_.nu / os_.de
    if OS == 1:
        OS = OS + 0.1
    fp = 1.0 / n_chan
    fs = 1.0 * (2 * OS - 1) / n_chan
    n_taps = n_chan * n_taps_per_chan
    return _firls(n_taps + 1, fp, fs)


def design_PFB_FIR_filter_two_stage(n_chan: int, os_factor, os_taps_per_chan: int = 28,
                                    zero_stuff_factor: int = None) -> np.ndarray:
    """design_PFB_FIR_filter_two_stage.m:19-84 — stage-1 firls of order n_taps/zsf, then
    zero-stuff its spectrum by zsf (returns n_taps + 1 taps, e.g. 100353 for Mid)."""
    os_ = as_rational(os_factor)
    osf = os_.nu / os_.de
    if zero_stuff_factor is None:
        zero_stuff_factor = (os_taps_per_chan * os_.nu) // os_.de if os_taps_per_chan != 28 else 32
    zsf = int(zero_stuff_factor)
    n_taps = int(round(os_taps_per_chan * n_chan / osf))
    n1 = n_taps // zsf
    fp = 1.0 / n_chan
    fs = (2 * osf - 1) / n_chan
    h0 = _firls(n1 + 1, fp * zsf, 0.998 * fs * zsf)
    H1 = np.fft.fft(np.fft.ifftshift(h0))
    # HZ = [H1(1:n1/2+1), zeros(1, n1*(zsf-1)), H1(n1/2+2:end)]
    HZ = np.concatenate([H1[:n1 // 2 + 1], np.zeros(n1 * (zsf - 1)), H1[n1 // 2 + 1:]])
    h = np.fft.fftshift(np.fft.ifft(HZ))
    return np.real(h)
