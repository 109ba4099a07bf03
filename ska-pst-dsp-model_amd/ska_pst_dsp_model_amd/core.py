"""Plans and the Matlab-shaped functional API of the PFB hot path.

    polyphase_analysis(in, filt, block, os_factor)          polyphase_analysis.m:1-7
    polyphase_analysis_padded(in, filt, block, os_factor)   polyphase_analysis_padded.m:1-7
    polyphase_synthesis(in, spans_nyq, Nf, os, deripple,
                        sample_offset, overlap, t_taper,
                        s_taper, combine)                    polyphase_synthesis.m:1-13

Arrays follow the Matlab shapes: analysis input (n_pol, 1, n_dat), channelised data
(n_pol, n_chan, n_dat), synthesis output (n_pol, 1, n_out).  Channelised arrays are
returned as a transposed *view* of a (n_pol, n_dat, n_chan) buffer — the per-pol
Matlab memory order (channel fastest), which is what the kernels read and write.

Inputs may be NumPy arrays (host; the C ABI stages them through device buffers) or
``torch`` tensors on a ROCm device (zero copy on the current stream).  Every call
goes through the HIP kernels of ``libpfb_hip.so``; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import hashlib
from ctypes import byref, c_int64, c_void_p

import numpy as np

from . import _lib
from .config import Rational, as_rational
from .window import PFBWindow, Taper, identity_taper

__all__ = ["AnalysisPlan", "SynthesisPlan", "polyphase_analysis", "polyphase_analysis_padded",
           "polyphase_analysis_lowcbf",
           "polyphase_synthesis", "analysis_plan", "synthesis_plan", "is_device_array",
           "roundtrip", "calc_output_nbins"]


def _torch():
    try:
        import torch  # noqa: F401
        return torch
    except Exception:  # pragma: no cover - torch is plumbing only
        return None


def is_device_array(x) -> bool:
    t = _torch()
    return t is not None and isinstance(x, t.Tensor) and x.is_cuda


def _stream_of(x, *plans):
    """The current stream of ``x``'s device as a C handle.  ``plans`` launched on it are
    marked when the stream is being captured into a graph (``close`` then refuses)."""
    t = _torch()
    s = t.cuda.current_stream(x.device)
    if plans and t.cuda.is_current_stream_capturing():
        for p in plans:
            p._capture_streams.append(s)
    return c_void_p(s.cuda_stream)


def _capturing(plan) -> bool:
    """Is a stream capture that recorded launches of ``plan`` still active?"""
    t = _torch()
    live = []
    for s in getattr(plan, "_capture_streams", ()):
        with t.cuda.stream(s):
            if t.cuda.is_current_stream_capturing():
                live.append(s)
    plan._capture_streams = live
    return bool(live)


def _close_guard(plan):
    # A captured graph references the plan's device buffers (taps, twiddles, stage-1 rows,
    # carry) by address: freeing them while the capture is open, or before every graph that
    # replays them is gone, makes the replays read freed memory.
    if getattr(plan, "_capture_streams", None) and _capturing(plan):
        raise RuntimeError(f"{type(plan).__name__}.close(): a stream capture that used this plan is "
                           "still active; end the capture (and drop its graphs) first")


def _taps64(filt) -> np.ndarray:
    if is_device_array(filt):
        filt = filt.detach().cpu().numpy()
    return np.ascontiguousarray(np.asarray(filt, dtype=np.float64).ravel())


# ============================================================================ analysis
class AnalysisPlan:
    """Device plan of one analysis filter bank (owns taps, twiddles, carry-over)."""

    def __init__(self, taps, n_chan: int, os_factor, variant: str = "polyphase_analysis",
                 n_pol: int = 1, device: int = 0):
        lib = _lib.load()
        _lib.require_device()
        self.os_factor = as_rational(os_factor)
        self.n_chan = int(n_chan)
        self.n_pol = int(n_pol)
        self.device = int(device)
        self.variant = variant
        v = {"polyphase_analysis": _lib.PFB_ANALYSIS_BUNTON, "bunton": _lib.PFB_ANALYSIS_BUNTON,
             "polyphase_analysis_padded": _lib.PFB_ANALYSIS_PADDED,
             "padded": _lib.PFB_ANALYSIS_PADDED,
             "polyphase_analysis_lowcbf": _lib.PFB_ANALYSIS_LOWCBF,
             "lowcbf": _lib.PFB_ANALYSIS_LOWCBF}
        if variant not in v:
            raise ValueError(f"unknown analysis function '{variant}'")
        self.taps = _taps64(taps)
        arr, ptr = _lib.c_double_array(self.taps)
        d = _lib.AnalysisDesc(v[variant], self.n_chan, self.os_factor.nu, self.os_factor.de,
                              ptr, len(arr), self.n_pol, self.device)
        h = c_void_p()
        _lib.check(lib.pfb_analysis_plan_create(byref(d), byref(h)))
        self._h = h
        self._capture_streams = []  # streams that captured launches of this plan
        self._lib = lib
        self.out_chan = int(lib.pfb_analysis_output_channels(h))  # 216 for LowCBF
        self.step = (self.n_chan * self.os_factor.de) // self.os_factor.nu
        self.phases = -(-len(self.taps) // self.n_chan)

    def close(self):
        if getattr(self, "_h", None):
            _close_guard(self)
            self._lib.pfb_analysis_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def output_length(self, n_dat: int) -> int:
        return int(self._lib.pfb_analysis_output_length(self._h, int(n_dat)))

    @property
    def buffered_samples(self) -> int:
        return int(self._lib.pfb_filterbank_buffered(self._h))

    def reset(self):
        _lib.check(self._lib.pfb_filterbank_reset(self._h))

    def stream_rows(self, n_in: int) -> int:
        """Rows the next stateful execute of n_in samples returns (nu-trimmed)."""
        return int(self._lib.pfb_filterbank_output_rows(self._h, int(n_in)))

    def execute_strided(self, x, out, out_pol_stride: int, row_stride: int, chan_stride: int,
                        sel=(0, 0, 0)):
        """Stateful execute of device series ``x`` (n_pol, n_dat; any pol stride, unit
        sample stride) writing bin c of row k of pol p to
        ``out``'s storage at p * out_pol_stride + k * row_stride + j * chan_stride
        (``pfb_filterbank_execute_strided``; sel = (split, shift, n) is the cascade's
        channel chomp).  Returns the number of rows written."""
        if x.shape[0] != self.n_pol or x.stride(1) != 1:
            raise ValueError("execute_strided: (n_pol, n_dat) series with unit sample stride")
        n_dat = int(x.shape[1])
        # elements of out's storage from its first element (the C ABI range-checks the
        # furthest strided write against it)
        cap = out.untyped_storage().nbytes() // out.element_size() - out.storage_offset()
        n_out = c_int64(0)
        _lib.check(self._lib.pfb_filterbank_execute_strided(
            self._h, c_void_p(x.data_ptr()), x.stride(0), n_dat, c_void_p(out.data_ptr()),
            int(out_pol_stride), int(row_stride), int(chan_stride), int(sel[0]), int(sel[1]),
            int(sel[2]), int(cap), byref(n_out), _stream_of(x, self)))
        return int(n_out.value)

    def _prep_in(self, x):
        """-> (array (n_pol, n_dat) complex64 contiguous, is_device)."""
        if is_device_array(x):
            t = _torch()
            x = x.to(t.complex64)
            if x.dim() == 3:
                x = x[:, 0, :]
            elif x.dim() == 1:
                x = x[None, :]
            x = x.contiguous()
            return x, True
        x = np.asarray(x)
        if x.ndim == 3:
            x = x[:, 0, :]
        elif x.ndim == 1:
            x = x[None, :]
        x = np.ascontiguousarray(x, dtype=np.complex64)
        return x, False

    def _alloc_out(self, like, dev, rows):
        if dev:
            t = _torch()
            return t.empty((self.n_pol, max(rows, 0), self.out_chan), dtype=t.complex64,
                           device=like.device)
        return np.empty((self.n_pol, max(rows, 0), self.out_chan), dtype=np.complex64)

    def execute(self, x, stateful: bool = False):
        """Run the analysis; returns the (n_pol, K, n_chan) buffer (time-major)."""
        x, dev = self._prep_in(x)
        if x.shape[0] != self.n_pol:
            raise ValueError(f"plan built for n_pol={self.n_pol}, got {x.shape[0]}")
        n_dat = x.shape[1]
        if stateful:
            cap = (self.buffered_samples + n_dat) // max(self.step, 1) + 1
        else:
            cap = self.output_length(n_dat)
        out = self._alloc_out(x, dev, cap)
        n_out = c_int64(0)
        if dev:
            src, dst, mem, stream = c_void_p(x.data_ptr()), c_void_p(out.data_ptr()), \
                _lib.PFB_MEM_DEVICE, _stream_of(x, self)
        else:
            src, dst, mem, stream = x.ctypes.data_as(c_void_p), out.ctypes.data_as(c_void_p), \
                _lib.PFB_MEM_HOST, c_void_p(0)
        fn = self._lib.pfb_filterbank_execute if stateful else self._lib.pfb_analysis_execute
        _lib.check(fn(self._h, src, n_dat, n_dat, dst, cap * self.out_chan, cap, byref(n_out),
                      mem, stream))
        return out[:, :n_out.value, :]


# ============================================================================ synthesis
def _resolve_taper(taper, nf: int, ov: int, spectral_length: int = 0):
    """Translate a taper handle into (kind, coeffs) for the C ABI.  ``spectral_length``
    > 0: the handle is a SPECTRAL taper over the L = spectral_length stitched bins
    (polyphase_synthesis.m:282); custom coefficients must then number L."""
    if taper is None or taper is identity_taper:
        return _lib.PFB_WINDOW_NONE, None
    if isinstance(taper, str):
        taper = PFBWindow().lookup[taper](nf, ov)
    if isinstance(taper, Taper) and spectral_length:
        if taper.kind == _lib.PFB_WINDOW_CUSTOM:
            c = np.asarray(taper.coeffs, dtype=np.float64).ravel()
            if c.size != spectral_length:
                raise ValueError(f"custom spectral taper needs {spectral_length} coefficients, "
                                 f"got {c.size}")
            return taper.kind, c
        return taper.kind, None  # hann: the plan builds circshift(hann(L), L/2)
    if isinstance(taper, Taper):
        if taper.kind == _lib.PFB_WINDOW_CUSTOM:
            return taper.kind, np.asarray(taper.coeffs, dtype=np.float64)
        if taper.kind in (_lib.PFB_WINDOW_TUKEY, _lib.PFB_WINDOW_TOP_HAT) and \
                (taper.input_fft_length, taper.input_discard) != (nf, ov):
            # the Matlab handle closes over its own (Nf, Ov); honour them explicitly
            return _lib.PFB_WINDOW_CUSTOM, taper.time_window(nf)
        return taper.kind, None
    kind = getattr(taper, "kind", None)
    if kind == _lib.PFB_WINDOW_NONE:
        return kind, None
    raise TypeError("polyphase_synthesis: arbitrary Python taper callables cannot run on the "
                    "GPU path; use a PFBWindow taper or PFBWindow().custom(coeffs)")


def _resolve_deripple(deripple):
    if deripple is None:
        return False, None
    if isinstance(deripple, dict):
        return bool(deripple.get("apply_deripple", 0)), deripple.get("filter_coeff")
    if isinstance(deripple, (tuple, list)):
        return bool(deripple[0]), deripple[1]
    if isinstance(deripple, (bool, int, np.bool_)):
        return bool(deripple), None
    return bool(getattr(deripple, "apply_deripple")), getattr(deripple, "filter_coeff", None)


class SynthesisPlan:
    """Device plan of one inverse filter bank (tables, twiddles, scratch, carry-over)."""

    def __init__(self, n_chan: int, os_factor, input_fft_length: int, input_overlap: int = None,
                 spans_nyquist: bool = True, combine: int = 1, deripple: bool = False,
                 filter_coeff=None, temporal_taper=None, spectral_taper=None, n_pol: int = 1,
                 device: int = 0):
        lib = _lib.load()
        _lib.require_device()
        self.os_factor = as_rational(os_factor)
        self.n_chan = int(n_chan)
        self.input_fft_length = int(input_fft_length)
        self.input_overlap = (self.input_fft_length // 8 if input_overlap is None
                              else int(input_overlap))
        self.n_pol = int(n_pol)
        self.device = int(device)
        nf, ov = self.input_fft_length, self.input_overlap
        tk, tco = _resolve_taper(temporal_taper, nf, ov)
        L = (nf * self.os_factor.de // self.os_factor.nu) * self.n_chan
        sk, sco = _resolve_taper(spectral_taper, nf, ov, spectral_length=L)
        taps = _taps64(filter_coeff) if filter_coeff is not None else np.zeros(1)
        self._keep = []
        tarr, tptr = _lib.c_double_array(taps)
        self._keep.append(tarr)
        tcp = sco_p = None
        if tco is not None:
            a, tcp = _lib.c_double_array(tco)
            self._keep.append(a)
        if sco is not None:
            a, sco_p = _lib.c_double_array(sco)
            self._keep.append(a)
        d = _lib.SynthesisDesc(self.n_chan, self.os_factor.nu, self.os_factor.de, nf, ov,
                               1 if spans_nyquist else 0, int(combine), 1 if deripple else 0,
                               tptr, len(tarr) if filter_coeff is not None else 0,
                               tk, tcp, sk, sco_p, self.n_pol, self.device)
        h = c_void_p()
        _lib.check(lib.pfb_synthesis_plan_create(byref(d), byref(h)))
        self._h = h
        self._capture_streams = []  # streams that captured launches of this plan
        self._lib = lib
        W = (nf * self.os_factor.de) // self.os_factor.nu
        self.output_fft_length = W * self.n_chan
        self.output_overlap = (ov * self.os_factor.de * self.n_chan) // self.os_factor.nu
        self.output_keep = self.output_fft_length - 2 * self.output_overlap
        self.input_keep = nf - 2 * ov

    def close(self):
        if getattr(self, "_h", None):
            _close_guard(self)
            self._lib.pfb_synthesis_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_chunk_blocks(self, blocks: int):
        _lib.check(self._lib.pfb_synthesis_set_chunk_blocks(self._h, int(blocks)))

    STAGE1_ROWS = {"auto": _lib.PFB_STAGE1_AUTO, "stored": _lib.PFB_STAGE1_STORED,
                   "recomputed": _lib.PFB_STAGE1_RECOMPUTED}

    def set_stage1_rows(self, mode: str):
        """Round trip only (pfb_synthesis_set_stage1_rows): 'stored' — the analysis writes
        the synthesis stage-1 rows and the synthesis reads them; 'recomputed' — the
        synthesis evaluates them from the input series (N = 256 streaming shapes;
        bit-identical output); 'auto' — the measured-faster one."""
        _lib.check(self._lib.pfb_synthesis_set_stage1_rows(self._h, self.STAGE1_ROWS[mode]))
        self._rt_input = None  # a split round trip in flight is not continued under another mode

    @property
    def last_stage1_rows(self) -> str:
        """Where the plan's last synthesis launch got its stage-1 rows ('stored',
        'recomputed'; 'none' before any launch) — pfb_synthesis_last_stage1_rows."""
        m = int(self._lib.pfb_synthesis_last_stage1_rows(self._h))
        return {_lib.PFB_STAGE1_STORED: "stored", _lib.PFB_STAGE1_RECOMPUTED: "recomputed"}.get(m, "none")

    def output_length(self, n_dat: int) -> int:
        return int(self._lib.pfb_synthesis_output_length(self._h, int(n_dat)))

    @property
    def buffered_samples(self) -> int:
        return int(self._lib.pfb_inverse_filterbank_buffered(self._h))

    def reset(self):
        _lib.check(self._lib.pfb_inverse_filterbank_reset(self._h))

    def set_stream_sample_offset(self, sample_offset: int):
        """InverseFilterBank.sample_offset (0-based) of the stateful ``execute(...,
        stateful=True)`` calls (pfb_inverse_filterbank_set_sample_offset)."""
        _lib.check(self._lib.pfb_inverse_filterbank_set_sample_offset(self._h, int(sample_offset)))

    def _prep_in(self, x, layout: str):
        """Accept (n_pol, n_chan, n_dat) Matlab-shaped or (n_pol, n_dat, n_chan) buffers."""
        if is_device_array(x):
            t = _torch()
            x = x.to(t.complex64)
            if layout == "pfc":
                ptc = x.transpose(1, 2)
            else:
                ptc = x
            return ptc.contiguous(), True
        x = np.asarray(x)
        ptc = x.transpose(0, 2, 1) if layout == "pfc" else x
        return np.ascontiguousarray(ptc, dtype=np.complex64), False

    def execute(self, x, sample_offset: int = 1, stateful: bool = False, layout: str = "pfc", out=None):
        """Run the synthesis; returns the (n_pol, n_out) series.  ``out``: an optional
        contiguous complex64 device buffer of at least (n_pol, output length) samples to
        write into (device input only; for graph capture without per-call allocations)."""
        ptc, dev = self._prep_in(x, layout)
        if ptc.shape[0] != self.n_pol or ptc.shape[2] != self.n_chan:
            raise ValueError(f"plan built for (n_pol={self.n_pol}, n_chan={self.n_chan}), "
                             f"got {tuple(ptc.shape)} [pol, time, chan]")
        n_dat = ptc.shape[1]
        if stateful:
            cap = self.output_length(self.buffered_samples + n_dat)
        else:
            cap = self.output_length(max(n_dat - (int(sample_offset) - 1), 0))
        if out is not None and not dev:
            raise ValueError("out= needs device input")
        if dev:
            t = _torch()
            if out is None:
                out = t.empty((self.n_pol, max(cap, 0)), dtype=t.complex64, device=ptc.device)
            elif (out.dtype != t.complex64 or out.device != ptc.device or not out.is_contiguous()
                  or out.dim() != 2 or out.shape[0] != self.n_pol or out.shape[1] < max(cap, 0)):
                raise ValueError(f"out must be a contiguous complex64 ({self.n_pol}, >= {max(cap, 0)}) "
                                 f"tensor on {ptc.device}, got {tuple(out.shape)} {out.dtype} {out.device}")
            cap = out.shape[1] if cap > 0 else cap
            src, dst, mem, stream = c_void_p(ptc.data_ptr()), c_void_p(out.data_ptr()), \
                _lib.PFB_MEM_DEVICE, _stream_of(ptc, self)
        else:
            out = np.empty((self.n_pol, max(cap, 0)), dtype=np.complex64)
            src, dst, mem, stream = ptc.ctypes.data_as(c_void_p), out.ctypes.data_as(c_void_p), \
                _lib.PFB_MEM_HOST, c_void_p(0)
        n_out = c_int64(0)
        if stateful:
            _lib.check(self._lib.pfb_inverse_filterbank_execute(
                self._h, src, n_dat * self.n_chan, n_dat, dst, cap, cap, byref(n_out), mem, stream))
        else:
            _lib.check(self._lib.pfb_synthesis_execute(
                self._h, src, n_dat * self.n_chan, n_dat, int(sample_offset), dst, cap, cap,
                byref(n_out), mem, stream))
        return out[:, :n_out.value]


# ============================================================================ round trip
def roundtrip(analysis: AnalysisPlan, synthesis: SynthesisPlan, x, sample_offset: int = 1,
              chan=None, out=None):
    """Analysis -> synthesis of ``x`` (device tensor, (n_pol, n_dat) or (n_pol, 1, n_dat))
    through ``pfb_roundtrip_execute`` — the sequence of test_data_pipeline.m:114,132.

    Returns ``(chan, out)``: the full channelised product as a (n_pol, K, n_chan)
    time-major buffer and the (n_pol, n_out) synthesised series.  ``chan`` is
    bit-identical to ``analysis.execute(x)``; ``out`` equals ``synthesis.execute(chan,
    sample_offset, layout="ptc")`` bit for bit on the chunked pipeline and to ~1e-7 on
    the fused path (include/pfb_api.h, pfb_roundtrip_execute).
    ``chan``/``out`` may be preallocated buffers of the right shapes (graph capture).
    """
    x, dev = analysis._prep_in(x)
    if not dev:
        raise ValueError("roundtrip() takes device tensors (use the separate calls for host arrays)")
    t = _torch()
    n_pol, n_dat = x.shape
    if n_pol != analysis.n_pol or n_pol != synthesis.n_pol:
        raise ValueError(f"plans built for n_pol={analysis.n_pol}/{synthesis.n_pol}, got {n_pol}")
    K = analysis.output_length(n_dat)
    n_out = synthesis.output_length(max(K - (int(sample_offset) - 1), 0))
    if chan is None:
        chan = t.empty((n_pol, max(K, 0), analysis.n_chan), dtype=t.complex64, device=x.device)
    if out is None:
        out = t.empty((n_pol, max(n_out, 0)), dtype=t.complex64, device=x.device)
    if tuple(chan.shape) != (n_pol, K, analysis.n_chan) or tuple(out.shape) != (n_pol, n_out):
        raise ValueError("preallocated chan/out have the wrong shape")
    kr, no = c_int64(0), c_int64(0)
    _lib.check(_lib.load().pfb_roundtrip_execute(
        analysis._h, synthesis._h, c_void_p(x.data_ptr()), n_dat, n_dat,
        c_void_p(chan.data_ptr()), K * analysis.n_chan, K, byref(kr), int(sample_offset),
        c_void_p(out.data_ptr()), max(n_out, 1), n_out, byref(no), _stream_of(x, analysis, synthesis)))
    return chan, out


def roundtrip_analysis(analysis: AnalysisPlan, synthesis: SynthesisPlan, x, sample_offset: int = 1,
                       chan=None):
    """The analysis half of the fused round trip (``pfb_roundtrip_analysis_execute``):
    writes the channelised product (returned, as ``roundtrip``'s ``chan``) and leaves the
    synthesis stage-1 rows in ``synthesis``'s scratch for ``roundtrip_synthesis``.  For
    pipelining consecutive blocks over two streams (each block on its own plan pair);
    the caller orders the halves.  ``PfbError`` (unsupported) when the plans take the
    chunked pipeline."""
    x, dev = analysis._prep_in(x)
    if not dev:
        raise ValueError("roundtrip_analysis() takes device tensors")
    t = _torch()
    n_pol, n_dat = x.shape
    if n_pol != analysis.n_pol or n_pol != synthesis.n_pol:
        raise ValueError(f"plans built for n_pol={analysis.n_pol}/{synthesis.n_pol}, got {n_pol}")
    K = analysis.output_length(n_dat)
    if chan is None:
        chan = t.empty((n_pol, max(K, 0), analysis.n_chan), dtype=t.complex64, device=x.device)
    if tuple(chan.shape) != (n_pol, K, analysis.n_chan):
        raise ValueError("preallocated chan has the wrong shape")
    kr = c_int64(0)
    _lib.check(_lib.load().pfb_roundtrip_analysis_execute(
        analysis._h, synthesis._h, c_void_p(x.data_ptr()), n_dat, n_dat,
        c_void_p(chan.data_ptr()), K * analysis.n_chan, K, byref(kr), int(sample_offset),
        _stream_of(x, analysis, synthesis)))
    # with recomputed stage-1 rows the synthesis half re-reads this input: `x` may be a
    # temporary made by _prep_in (another dtype, a non-contiguous view), so the plan keeps
    # it alive until roundtrip_synthesis has been enqueued (which records it on its stream)
    synthesis._rt_input = x
    return chan


def roundtrip_synthesis(analysis: AnalysisPlan, synthesis: SynthesisPlan, n_dat: int,
                        sample_offset: int = 1, out=None, device=None):
    """The synthesis half (``pfb_roundtrip_synthesis_execute``) of a
    ``roundtrip_analysis`` call with the same ``n_dat`` / ``sample_offset``: returns the
    (n_pol, n_out) series, equal to ``roundtrip``'s ``out`` bit for bit.  Runs on the
    current stream of ``out``'s device (or ``device``)."""
    t = _torch()
    n_pol = synthesis.n_pol
    K = analysis.output_length(int(n_dat))
    n_out = synthesis.output_length(max(K - (int(sample_offset) - 1), 0))
    if out is None:
        dv = t.device("cuda", synthesis.device if device is None else device)
        out = t.empty((n_pol, max(n_out, 0)), dtype=t.complex64, device=dv)
    if tuple(out.shape) != (n_pol, n_out):
        raise ValueError("preallocated out has the wrong shape")
    no = c_int64(0)
    stream = _stream_of(out, analysis, synthesis)
    _lib.check(_lib.load().pfb_roundtrip_synthesis_execute(
        analysis._h, synthesis._h, int(n_dat), int(sample_offset), c_void_p(out.data_ptr()),
        max(n_out, 1), n_out, byref(no), stream))
    xin = getattr(synthesis, "_rt_input", None)
    if xin is not None:
        # the analysis half's input (recomputed rows read it here): its memory may be reused
        # only after the work just enqueued on this stream has finished
        if not t.cuda.is_current_stream_capturing():
            xin.record_stream(t.cuda.current_stream(out.device))
        else:
            # a captured launch holds the input's address for every replay: keep the tensor
            # alive as long as the plan (one entry per address, so recaptures do not grow it)
            held = synthesis.__dict__.setdefault("_graph_inputs", {})
            held[xin.data_ptr()] = xin
        synthesis._rt_input = None
    return out


# ============================================================================ helpers
def calc_output_nbins(nbins, channels, os_factor, filter_taps, input_fft_length, input_overlap):
    """calc_output_nbins.m:1-28 (same arguments: ``os_factor`` a Rational / "nu/de" / Matlab
    struct-like, ``filter_taps`` the tap COUNT): the number of samples that emerge from
    channelisation and inversion of ``nbins`` input samples.  Evaluated by the C ABI
    (``pfb_calc_output_nbins``) in Matlab's double arithmetic; integral results come
    back as int."""
    os_ = as_rational(os_factor)
    v = float(_lib.load().pfb_calc_output_nbins(int(nbins), int(channels), os_.nu, os_.de,
                                                int(filter_taps), int(input_fft_length),
                                                int(input_overlap)))
    return int(v) if v.is_integer() else v


# ============================================================================ plan cache
_PLANS = {}


def _key(*parts):
    h = hashlib.sha1()
    for p in parts:
        if isinstance(p, np.ndarray):
            h.update(p.tobytes())
        else:
            h.update(repr(p).encode())
    return h.hexdigest()


def analysis_plan(filt, block, os_factor, variant, n_pol, device=0) -> AnalysisPlan:
    taps = _taps64(filt)
    os_ = as_rational(os_factor)
    k = _key("a", taps, int(block), str(os_), variant, int(n_pol), int(device))
    p = _PLANS.get(k)
    if p is None:
        p = AnalysisPlan(taps, block, os_, variant, n_pol, device)
        _PLANS[k] = p
    return p


def synthesis_plan(n_chan, os_factor, nf, ov, spans, combine, deripple, filt, t_taper, s_taper,
                   n_pol, device=0) -> SynthesisPlan:
    os_ = as_rational(os_factor)
    tk, tco = _resolve_taper(t_taper, nf, ov)
    sk, sco = _resolve_taper(s_taper, nf, ov, spectral_length=(nf * os_.de // os_.nu) * int(n_chan))
    taps = _taps64(filt) if (deripple and filt is not None) else None
    k = _key("s", int(n_chan), str(os_), int(nf), int(ov), bool(spans), int(combine),
             bool(deripple), taps if taps is not None else "-", tk,
             tco if tco is not None else "-", sk, sco if sco is not None else "-",
             int(n_pol), int(device))
    p = _PLANS.get(k)
    if p is None:
        p = SynthesisPlan(n_chan, os_, nf, ov, spans, combine, deripple, taps, t_taper, s_taper,
                          n_pol, device)
        _PLANS[k] = p
    return p


def _device_of(x) -> int:
    if is_device_array(x):
        return x.device.index or 0
    return 0


def _pfc_view(buf):
    """(n_pol, K, N) buffer -> Matlab-shaped (n_pol, N, K) view."""
    if is_device_array(buf):
        return buf.transpose(1, 2)
    return buf.transpose(0, 2, 1)


def _npol(x) -> int:
    shape = tuple(x.shape)
    return 1 if len(shape) == 1 else int(shape[0])


# ============================================================================ functions
def polyphase_analysis(in_, filt, block, os_factor, verbose_=0):
    """polyphase_analysis.m:1-129 (Bunton).  Returns (n_pol, block, nblocks) complex64."""
    plan = analysis_plan(filt, block, os_factor, "polyphase_analysis", _npol(in_),
                         _device_of(in_))
    return _pfc_view(plan.execute(in_))


def polyphase_analysis_padded(in_, filt, block, os_factor, verbose_=0):
    """polyphase_analysis_padded.m:1-161 (commutator).  Returns (n_pol, block, nblocks)."""
    plan = analysis_plan(filt, block, os_factor, "polyphase_analysis_padded", _npol(in_),
                         _device_of(in_))
    return _pfc_view(plan.execute(in_))


def polyphase_analysis_lowcbf(in_, filt, block=256, os_factor="4/3", verbose_=0):
    """polyphase_analysis_lowcbf.m:1-49 (SKA-Low CBF PST filterbank, PSTFilterbank.m).
    Returns (n_pol, 216, nblocks).  The wrapper's ``persistent do_padding`` (1536 zeros
    before the first call's data only) lives in the cached plan of these taps."""
    plan = analysis_plan(filt, 256, "4/3", "polyphase_analysis_lowcbf", _npol(in_),
                         _device_of(in_))
    return _pfc_view(plan.execute(in_))


def polyphase_synthesis(in_, input_fully_spans_Nyquist_zone, input_fft_length, os_factor,
                        deripple_=None, sample_offset_=1, input_overlap_=None,
                        temporal_taper_=None, spectral_taper_=None, combine_=1, verbose_=0):
    """polyphase_synthesis.m:1-325 (golden inversion).  Returns (n_pol, 1, n_out)."""
    nf = int(input_fft_length)
    ov = nf // 8 if input_overlap_ is None else int(input_overlap_)
    dr, filt = _resolve_deripple(deripple_)
    shape = tuple(in_.shape)
    if len(shape) != 3:
        raise ValueError("polyphase_synthesis input must be (n_pol, n_chan, n_dat)")
    if not is_device_array(in_) and not np.iscomplexobj(np.asarray(in_)):
        raise ValueError("polyphase_synthesis input data are real-valued!")
    plan = synthesis_plan(shape[1], os_factor, nf, ov, bool(input_fully_spans_Nyquist_zone),
                          int(combine_), dr, filt, temporal_taper_, spectral_taper_, shape[0],
                          _device_of(in_))
    out = plan.execute(in_, sample_offset=int(sample_offset_))
    return out[:, None, :]
