"""Device data-format operations of the C ABI (``pfb_layout.hip``): DADA unpack/pack,
corner turn, channel gather and the FilterBank quantisation hook.

Every function takes and returns ROCm ``torch`` tensors (device memory; torch is only
the allocator and stream here) and runs one hand-written HIP kernel on the tensor's
current stream.  There is no CPU path: host arrays must be moved to the device first.
"""
from __future__ import annotations

from ctypes import byref, c_double, c_void_p

from . import _lib

__all__ = ["dada_unpack", "dada_pack", "corner_turn", "gather_channels", "quantize",
           "nbit_dtype"]


def _torch():
    import torch
    return torch


def _stream(t):
    return c_void_p(_torch().cuda.current_stream(t.device).cuda_stream)


def _require_device(x, name):
    torch = _torch()
    if not (isinstance(x, torch.Tensor) and x.is_cuda):
        raise _lib.PfbError(_lib.PFB_ERR_INVALID_ARG, f"{name}: expects a device tensor")


def nbit_dtype(nbit: int):
    """Sample type of a DADA NBIT value (DADARead.m:49-55)."""
    torch = _torch()
    return {8: torch.int8, 16: torch.int16, 32: torch.float32, 64: torch.float64}[int(nbit)]


def dada_unpack(raw, nbit: int, ndim: int, n_chan: int, n_pol: int, lowcbf: bool = False):
    """DADA data section (device tensor of bytes or samples) -> (n_pol, n_dat, n_chan)
    complex64 — ``reshape_dada_data.m`` / ``reshape_low_cbf_data.m`` + the cast of
    ``DADARead.m:68-72``.  n_dat is inferred from the size (trailing partial samples,
    or a partial LowCBF heap, are dropped like ``fread`` + ``reshape`` would refuse)."""
    torch = _torch()
    _require_device(raw, "dada_unpack")
    nbytes = raw.numel() * raw.element_size()
    per = n_chan * n_pol * ndim * (nbit // 8)
    n_dat = nbytes // per
    if lowcbf:
        n_dat -= n_dat % 32
    out = torch.empty((n_pol, n_dat, n_chan), dtype=torch.complex64, device=raw.device)
    lib = _lib.load()
    _lib.check(lib.pfb_dada_unpack(c_void_p(raw.data_ptr()), int(nbit), int(ndim),
                                   _lib.PFB_DADA_LOWCBF if lowcbf else _lib.PFB_DADA_TFP,
                                   int(n_dat), int(n_chan), int(n_pol), c_void_p(out.data_ptr()),
                                   int(n_dat * n_chan), _stream(raw)))
    return out


def dada_pack(x, nbit: int = 32):
    """(n_pol, n_dat, n_chan) complex64 device tensor -> 1-D device tensor of the TFP
    data section in the sample type of ``nbit`` (``write_dada_data.m:32-50``)."""
    torch = _torch()
    _require_device(x, "dada_pack")
    x = x.to(torch.complex64).contiguous()
    n_pol, n_dat, n_chan = (int(s) for s in x.shape)
    out = torch.empty((n_dat * n_chan * n_pol * 2,), dtype=nbit_dtype(nbit),
                      device=x.device)
    _lib.check(_lib.load().pfb_dada_pack(c_void_p(x.data_ptr()), n_dat * n_chan, n_dat, n_chan,
                                         n_pol, c_void_p(out.data_ptr()), int(nbit), _stream(x)))
    return out


def corner_turn(x):
    """(B, R, C) -> (B, C, R) contiguous (``pfb_corner_turn``); 2-D inputs are B = 1."""
    torch = _torch()
    _require_device(x, "corner_turn")
    squeeze = x.dim() == 2
    if squeeze:
        x = x[None]
    if x.stride(2) != 1:
        x = x.contiguous()
    B, R, C = (int(s) for s in x.shape)
    out = torch.empty((B, C, R), dtype=torch.complex64, device=x.device)
    _lib.check(_lib.load().pfb_corner_turn(c_void_p(x.data_ptr()), x.stride(0), x.stride(1), B, R,
                                           C, c_void_p(out.data_ptr()), C * R, R, _stream(x)))
    return out[0] if squeeze else out


def gather_channels(x, n_outer: int, in_outer_stride: int, in_row_stride: int, n_rows: int,
                    n_sel: int, src0: int = 0, split: int = None, shift: int = 0, out=None,
                    out_outer_stride: int = None, out_row_stride: int = None):
    """out[o, t, j] = x[o*ios + t*irs + src0 + j + (j >= split ? shift : 0)] (flat complex
    sample offsets into ``x``'s storage) — ``pfb_gather_channels``.  Without ``out`` the
    result is a new (n_outer, n_rows, n_sel) tensor."""
    torch = _torch()
    _require_device(x, "gather_channels")
    if out is None:
        out = torch.empty((n_outer, n_rows, n_sel), dtype=torch.complex64, device=x.device)
        out_outer_stride, out_row_stride = n_rows * n_sel, n_sel
    split = n_sel if split is None else int(split)
    _lib.check(_lib.load().pfb_gather_channels(
        c_void_p(x.data_ptr()), int(in_outer_stride), int(in_row_stride), c_void_p(out.data_ptr()),
        int(out_outer_stride), int(out_row_stride), int(n_outer), int(n_rows), int(n_sel),
        int(src0), split, int(shift), _stream(x)))
    return out


def quantize(x, rms: float = 0.0, out=None, return_scale: bool = False):
    """round(single(rms / std(x)) * x) (or round(x) for rms <= 0) over the whole
    (n_pol, ...) array — FilterBank.m:75-83,106-113 — in one device reduction plus one
    rounding pass (``pfb_quantize``).  ``x`` is viewed as (n_pol, n) rows."""
    torch = _torch()
    _require_device(x, "quantize")
    src = x.to(torch.complex64)
    shape = tuple(src.shape)
    n_pol = shape[0] if len(shape) > 1 else 1
    flat = src.reshape(n_pol, -1)
    if flat.stride(1) != 1:
        flat = flat.contiguous()
    n = int(flat.shape[1])
    if out is None:
        out = torch.empty((n_pol, n), dtype=torch.complex64, device=x.device)
    sc = c_double(1.0)
    _lib.check(_lib.load().pfb_quantize(c_void_p(flat.data_ptr()), flat.stride(0), n, n_pol,
                                        float(rms), c_void_p(out.data_ptr()), out.stride(0),
                                        byref(sc) if return_scale else None, _stream(flat)))
    res = out.reshape(shape)
    return (res, sc.value) if return_scale else res
