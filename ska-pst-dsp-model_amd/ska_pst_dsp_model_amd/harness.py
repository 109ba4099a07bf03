"""The Python harness' backend switch with a ``"hip"`` backend.

Mirrors ``python/data_gen``: ``channelize`` (channelize.py:19-92), ``synthesize``
(synthesize.py:27-95), ``pipeline`` (pipeline.py:13-86) and ``generate_test_vector``
(generate_test_vector.py:24-209) with the same call shapes, returning DADA file objects
(``dada.DADAFile``).  The file semantics are those of the compiled Matlab commands the
``"matlab"`` backend runs: ``channelize.m`` (header TSAMP / PFB_DC_CHAN / NCHAN_PFB_0 /
OS_FACTOR / FIR coefficients, ``add_fir_filter_to_header.m``) and ``synthesize.m``
(NCHAN / OS_FACTOR / COEFF_0 read back from the header, TSAMP rescaled).  The data
never visit the host between the file read and the file write: DADA unpack, analysis
or synthesis and DADA pack all run on the device.

Only ``backend="hip"`` is provided: the reference's ``"matlab"`` (compiled MCR
binaries) and ``"python"`` (the un-vendored ``pfb`` package) backends are absent here.
"""
from __future__ import annotations

import functools
import os

import numpy as np

from . import dada
from .config import as_rational
from .core import polyphase_analysis, polyphase_analysis_padded, polyphase_synthesis
from .firio import read_fir_filter_coeff
from .window import PFBWindow

__all__ = ["channelize", "synthesize", "pipeline", "generate_test_vector", "complex_sinusoid",
           "time_domain_impulse", "create_output_file_names"]


def _check_backend(backend):
    if backend != "hip":
        raise ValueError(f"backend '{backend}' is not available; this engine provides 'hip'")


def create_output_file_names(output_file_name, default_base):
    """data_gen/util.py:94-102."""
    if output_file_name is None:
        output_base = default_base
        output_file_name = output_base + ".dump"
    else:
        output_base = os.path.splitext(output_file_name)[0]
    return output_base, output_base + ".log", output_file_name


def _num2str(v: float) -> str:
    """Matlab num2str of a real scalar: integers as %d, otherwise %.{d+4}g with d the
    number of integer digits (at least 1)."""
    if v == int(v):
        return str(int(v))
    d = max(1, int(np.floor(np.log10(abs(v)))) + 1)
    return ("%%.%dg" % (d + 4)) % v


def channelize(input_data_file_path: str, channels: int = None, os_factor_str: str = None,
               fir_filter_path: str = None, output_file_name: str = None,
               output_dir: str = "./", backend: str = "hip", use_padded: bool = False,
               device: int = 0):
    """channelize.py:19-92 / channelize.m:1-113 on the HIP engine."""
    _check_backend(backend)
    if channels is None or os_factor_str is None or fir_filter_path is None:
        raise ValueError("channelize: channels, os_factor_str and fir_filter_path are required")
    os_factor = as_rational(str(os_factor_str))
    output_base = f"channelize.{channels}.{'-'.join(str(os_factor_str).split('/'))}"
    _, _, output_file_name = create_output_file_names(output_file_name, output_base)
    data, hdr = dada.read_dada_file(input_data_file_path, device)
    taps = read_fir_filter_coeff(fir_filter_path)
    ch = dict(hdr)
    tsamp = float(hdr.get("TSAMP", "1"))
    ch["TSAMP"] = _num2str(tsamp * os_factor.de / os_factor.nu * channels)  # channelize.m:75
    ch["PFB_DC_CHAN"] = "1"
    ch["NCHAN_PFB_0"] = str(int(channels))
    ch["OS_FACTOR"] = f"{os_factor.nu}/{os_factor.de}"
    dada.add_fir_filter_to_header(ch, taps, os_factor)
    fn = polyphase_analysis_padded if use_padded else polyphase_analysis
    chan = fn(data[:, 0, :], taps, int(channels), os_factor)  # (n_pol, channels, K)
    path = os.path.join(output_dir, output_file_name)
    dada.write_dada_file(path, chan, ch)
    return dada.DADAFile(path, device).load_data()


def synthesize(input_data_file_path, input_fft_length: int = None, input_overlap: int = None,
               fft_window_str: str = "no_window", output_file_name: str = None,
               output_dir: str = "./", deripple: bool = True, backend: str = "hip",
               device: int = 0):
    """synthesize.py:27-95 / synthesize.m:1-119 on the HIP engine (spans-Nyquist golden
    inversion, sample_offset 1; FIR taps for the deripple from the header's COEFF_0,
    i.e. at the '%0.6E' precision the channelizer wrote them)."""
    _check_backend(backend)
    if input_fft_length is None or input_overlap is None:
        raise ValueError("synthesize: input_fft_length and input_overlap are required")
    nf, ov = int(input_fft_length), int(input_overlap)
    output_base = f"synthesize.{nf}"
    _, _, output_file_name = create_output_file_names(output_file_name, output_base)
    data, hdr = dada.read_dada_file(input_data_file_path, device)
    channels = int(hdr["NCHAN"])
    os_factor = as_rational(hdr["OS_FACTOR"])
    taps = np.array([float(v) for v in hdr["COEFF_0"].split(",")])
    taper = PFBWindow().lookup[fft_window_str](nf, ov)
    sh = dict(hdr)
    tsamp = float(hdr.get("TSAMP", "1"))
    sh["TSAMP"] = _num2str(tsamp / (os_factor.de / os_factor.nu) / channels)
    out = polyphase_synthesis(data, 1, nf, os_factor,
                              {"apply_deripple": int(bool(deripple)), "filter_coeff": taps}, 1,
                              ov, taper)
    path = os.path.join(output_dir, output_file_name)
    dada.write_dada_file(path, out, sh)
    return dada.DADAFile(path, device).load_data()


def pipeline(test_vector_callback, channelize_callback, synthesize_callback, output_dir=None):
    """pipeline.py:13-86: generate -> channelize -> synthesize, each step a DADA file."""
    def _pipeline(*args, **kwargs):
        tv = test_vector_callback(*args, **kwargs, output_dir=output_dir)
        base = os.path.basename(tv.file_path)
        ch = channelize_callback(tv.file_path, output_file_name="channelized." + base,
                                 output_dir=output_dir)
        sy = synthesize_callback(ch.file_path, output_file_name="synthesized." + base,
                                 output_dir=output_dir)
        return tv, ch, sy
    return _pipeline


def complex_sinusoid(n: int, freqs, phases, bin_offset: float = 0.0, dtype=np.complex64):
    """generate_test_vector.py:24-48."""
    if not hasattr(freqs, "__iter__"):
        freqs, phases = [freqs], [phases]
    t = np.arange(n)
    sig = np.zeros(n, dtype=dtype)
    for f, ph in zip(freqs, phases):
        if f < 1.0:
            f = int(n * f)
        sig += np.exp(1j * (2 * np.pi * (f + bin_offset) / n * t + ph))
    return sig


def time_domain_impulse(n: int, offsets, widths, dtype=np.complex64):
    """generate_test_vector.py:51-70."""
    if not hasattr(offsets, "__iter__"):
        offsets, widths = [offsets], [widths]
    sig = np.zeros(n, dtype=dtype)
    for off, w in zip(offsets, widths):
        if off < 1.0:
            off = int(off * n)
        sig[off:off + w] = 1.0
    return sig


_DEFAULT_HEADER = {"HDR_VERSION": "1.0", "HDR_SIZE": "4096", "INSTRUMENT": "dspsr",
                   "TELESCOPE": "PKS", "SOURCE": "TestVector", "TSAMP": "1", "FREQ": "1405",
                   "BW": "40", "OBS_OFFSET": "0", "UTC_START": "2019-02-05-01:15:49"}


def generate_test_vector(*args, n_bins: int, domain_name: str, header_template: dict = None,
                         output_file_name: str = None, output_dir: str = "./", n_pol: int = 1,
                         dtype=np.complex64, backend: str = "hip", device: int = 0):
    """generate_test_vector.py:73-209 (``python`` branch semantics: the signal repeated
    over n_pol, written as a single-channel DADA file)."""
    _check_backend(backend)
    funcs = {"time": time_domain_impulse, "freq": complex_sinusoid}
    sig = funcs[domain_name](n_bins, *args, dtype=dtype)
    arg_str = "-".join(f"{(a[0] if hasattr(a, '__iter__') else a):.3f}" for a in args)
    base = f"{funcs[domain_name].__name__}.{n_bins}.{arg_str}.{n_pol}.single.{backend}"
    _, _, output_file_name = create_output_file_names(output_file_name, base)
    data = np.repeat(sig.astype(np.complex64)[None, None, :], n_pol, axis=0)
    path = os.path.join(output_dir, output_file_name)
    dada.write_dada_file(path, data, dict(header_template or _DEFAULT_HEADER))
    return dada.DADAFile(path, device).load_data()


def partial(fn, **kw):
    """``partialize`` stand-in: pre-bind keyword arguments (channelize(backend=...))."""
    return functools.partial(fn, **kw)
