"""DADA file I/O with on-device unpack/pack.

Host side (this module): the ASCII header — ``read_header.m:12-39`` (4096-byte
default, ``HDR_SIZE`` re-read, ``#`` comments, first two whitespace tokens of a line)
and ``write_header.m:8-48`` (``HDR_SIZE`` first, remaining keys in
``containers.Map`` order = sorted, NUL padding, size doubled when it does not fit) —
and the raw byte transfer.  Device side (``pfb_dada_unpack`` / ``pfb_dada_pack``): the
TFP <-> [pol][t][chan] reordering and sample-type conversion of
``reshape_dada_data.m``, ``reshape_low_cbf_data.m``, ``DADARead.m:58-83`` and
``write_dada_data.m:32-50``.  Only the file's raw bytes cross PCIe (an NBIT 8 file
moves 2 bytes per complex sample instead of 8).

Arrays follow the Matlab shapes: ``read_dada_file`` returns ``(n_pol, n_chan, n_dat)``
(a view of the engine's (n_pol, n_dat, n_chan) buffer), ``write_dada_file`` takes the
same.
"""
from __future__ import annotations

import os
import re

import numpy as np

from . import layout

__all__ = ["read_header", "write_header", "read_dada_file", "write_dada_file",
           "write_dada_header", "DADARead", "DADAWrite", "DADAFile", "add_fir_filter_to_header"]

_NBIT_NP = {8: np.int8, 16: np.int16, 32: np.float32, 64: np.float64}


def _torch():
    import torch
    return torch


# ------------------------------------------------------------------ header
_WS = re.compile(r"[ \f\n\r\t\v]+")


def _parse_header(text: str) -> dict:
    """read_header.m:16-27: lines split at '\n'; '#' lines skipped; strsplit(line) at
    collapsed whitespace (a leading or trailing run gives an empty first or last token, as
    in Matlab); a line with more than one token maps token 1 -> token 2.  The text ends at
    the first NUL (the header padding; read_header.m would store that padding under an
    empty key)."""
    hdr = {}
    for line in text.split("\n"):
        if line.startswith("#"):
            continue
        tok = _WS.split(line)
        if len(tok) > 1:
            hdr[tok[0]] = tok[1]
    return hdr


def read_header(f) -> dict:
    """read_header.m:12-39 — ``f`` is a path or a binary file object."""
    if isinstance(f, (str, os.PathLike)):
        with open(f, "rb") as fh:
            return read_header(fh)
    size = 4096
    for _ in range(32):
        f.seek(0)
        raw = f.read(size)
        text = raw.split(b"\0", 1)[0].decode("ascii", errors="replace")
        hdr = _parse_header(text)
        if "HDR_SIZE" in hdr:
            new = int(float(hdr["HDR_SIZE"]))
            if new == size:
                return hdr
            size = new
        else:
            if len(raw) < size:  # whole file read and no HDR_SIZE: give up like fscanf would
                return hdr
            size *= 2
    raise ValueError("read_header: HDR_SIZE does not converge")


def _header_text(hdr: dict) -> str:
    s = f"HDR_SIZE {hdr['HDR_SIZE']}\n"
    for k in sorted(hdr):  # containers.Map iterates keys in sorted order
        if k == "HDR_SIZE":
            continue
        s += f"{k} {hdr[k]}\n"
    return s


def write_header(f, hdr: dict) -> None:
    """write_header.m:8-48: HDR_SIZE line first, NUL-padded to HDR_SIZE bytes."""
    hdr = dict(hdr)
    hdr.setdefault("HDR_SIZE", "4096")
    text = _header_text(hdr)
    while len(text) > int(hdr["HDR_SIZE"]):
        hdr["HDR_SIZE"] = str(int(hdr["HDR_SIZE"]) * 2)
        text = _header_text(hdr)
    size = int(hdr["HDR_SIZE"])
    f.seek(0)
    f.write(text.encode("ascii") + b"\0" * (size - len(text)))
    if f.tell() != size:
        raise IOError("Incorrect file pointer after writing header")


def add_fir_filter_to_header(hdr: dict, fir_filter_coeff, os_factors) -> dict:
    """add_fir_filter_to_header.m:1-40 (coefficients printed '%0.6E')."""
    from .config import as_rational
    firs = fir_filter_coeff if isinstance(fir_filter_coeff, (list, tuple)) else [fir_filter_coeff]
    oss = os_factors if isinstance(os_factors, (list, tuple)) else [os_factors]
    hdr["NSTAGE"] = str(len(firs))
    for n, (fir, os_) in enumerate(zip(firs, oss)):
        fir = np.asarray(fir, dtype=np.float64).ravel()
        o = as_rational(os_)
        hdr[f"COEFF_{n}"] = ",".join("%0.6E" % v for v in fir)
        hdr[f"OVERSAMP_{n}"] = f"{o.nu}/{o.de}"
        hdr[f"NTAP_{n}"] = str(len(fir))
    return hdr


# ------------------------------------------------------------------ data
def _device(device):
    torch = _torch()
    if isinstance(device, torch.device):
        return device
    return torch.device("cuda", int(device))


def _to_device_raw(buf: np.ndarray, device):
    torch = _torch()
    t = torch.from_numpy(np.ascontiguousarray(buf).view(np.uint8))
    return t.to(_device(device), non_blocking=False)


def _unpack(raw_dev, hdr: dict, lowcbf: bool):
    nbit = int(hdr["NBIT"])
    ndim = int(hdr["NDIM"])
    npol = int(hdr["NPOL"])
    nchan = int(hdr["NCHAN"])
    return layout.dada_unpack(raw_dev, nbit, ndim, nchan, npol, lowcbf=lowcbf)


def _matlab_view(buf):
    return buf.transpose(1, 2)  # (n_pol, n_dat, n_chan) -> (n_pol, n_chan, n_dat)


def read_dada_file(path, device=0):
    """read_dada_file.m:1-48 -> ``(data, header)``; ``data`` is a (n_pol, n_chan, n_dat)
    complex64 device tensor (view of the (n_pol, n_dat, n_chan) engine buffer)."""
    with open(path, "rb") as f:
        hdr = read_header(f)
        f.seek(int(hdr["HDR_SIZE"]))
        raw = np.fromfile(f, dtype=np.uint8)
    lowcbf = hdr.get("INSTRUMENT") == "LowCBF"
    if lowcbf:
        raise ValueError("read_dada_file: LowCBF files are read with DADARead "
                         "(read_dada_file.m has no heap reordering)")
    return _matlab_view(_unpack(_to_device_raw(raw, device), hdr, False)), hdr


def write_dada_header(f, data_shape, nbit: int, hdr: dict, ndim: int = 2) -> dict:
    """write_dada_header.m:1-26 (NBIT from the data class, NDIM 2 for complex data,
    NPOL/NCHAN from the Matlab (n_pol, n_chan, n_dat) shape)."""
    h = dict(hdr)
    h["NBIT"] = str(int(nbit))
    h["NDIM"] = str(int(ndim))
    h["NPOL"] = str(int(data_shape[0]))
    h["NCHAN"] = str(int(data_shape[1]))
    write_header(f, h)
    return h


def _pack_to_host(data, nbit: int) -> np.ndarray:
    """(n_pol, n_chan, n_dat) device tensor -> host bytes of the TFP data section."""
    torch = _torch()
    buf = data.transpose(1, 2)  # engine (n_pol, n_dat, n_chan) order
    if not buf.is_contiguous():
        buf = buf.contiguous()
    packed = layout.dada_pack(buf.to(torch.complex64), nbit)
    return packed.cpu().numpy()


def write_dada_file(path, data, hdr: dict, nbit: int = 32) -> dict:
    """write_dada_file.m:1-25: header (write_dada_header) then data (write_dada_data).
    ``data`` is a Matlab-shaped (n_pol, n_chan, n_dat) complex array (device tensor or
    NumPy; NumPy arrays are moved to device 0 for the pack kernel)."""
    torch = _torch()
    if not (isinstance(data, torch.Tensor) and data.is_cuda):
        data = torch.from_numpy(np.ascontiguousarray(np.asarray(data, dtype=np.complex64))).cuda()
    if data.dim() != 3:
        raise ValueError("write_dada_file: data must be (n_pol, n_chan, n_dat)")
    with open(path, "wb") as f:
        h = write_dada_header(f, tuple(data.shape), nbit, hdr)
        body = _pack_to_host(data, nbit)
        f.write(body.tobytes())
    return h


class DADARead:
    """DADARead.m:1-85 — streaming reader; ``generate(nsample)`` returns the next
    nsample samples as a (n_pol, n_chan, nsample) complex64 device tensor."""

    def __init__(self, device=0):
        self.filename = ""
        self.header = {}
        self.n_dim = self.n_pol = self.n_chan = self.n_bit = 1
        self.low_cbf_input = False
        self.device = device
        self._f = None

    def open(self, fname):
        self._f = open(fname, "rb")
        self.header = read_header(self._f)
        self._f.seek(int(self.header["HDR_SIZE"]))
        self.low_cbf_input = self.header.get("INSTRUMENT") == "LowCBF"
        self.n_dim = int(self.header["NDIM"])
        self.n_pol = int(self.header["NPOL"])
        self.n_bit = int(self.header["NBIT"])
        self.n_chan = int(self.header["NCHAN"])
        self.filename = str(fname)
        return self

    def generate(self, nsample: int):
        nbytes = nsample * self.n_chan * self.n_pol * self.n_dim * (self.n_bit // 8)
        raw = np.fromfile(self._f, dtype=np.uint8, count=nbytes)
        dev = _to_device_raw(raw, self.device)
        return self, _matlab_view(_unpack(dev, self.header, self.low_cbf_input))

    def close(self):
        if self._f:
            self._f.close()
            self._f = None
        return self


class DADAWrite:
    """DADAWrite.m:1-50 — header on the first write, then data appended."""

    def __init__(self, filename="", header=None, nbit: int = 32):
        self.filename = filename
        self.header = dict(header or {})
        self.nbit = nbit
        self._f = None

    def open(self, fname):
        self._f = open(fname, "wb")
        self.filename = str(fname)
        return self

    def write(self, data):
        torch = _torch()
        if not (isinstance(data, torch.Tensor) and data.is_cuda):
            data = torch.from_numpy(np.ascontiguousarray(np.asarray(data, dtype=np.complex64))).cuda()
        if self._f is None:
            self.open(self.filename)
        if self._f.tell() == 0:
            write_dada_header(self._f, tuple(data.shape), self.nbit, self.header)
        self._f.write(_pack_to_host(data, self.nbit).tobytes())
        return self

    def close(self):
        if self._f:
            self._f.close()
            self._f = None
        return self


class DADAFile:
    """The ``psr_formats.DADAFile`` surface the Python harness passes around
    (``file_path``, ``header``, ``data`` as (n_dat, n_chan, n_pol) host array,
    ``load_data()``)."""

    def __init__(self, file_path, device=0):
        self.file_path = str(file_path)
        self.header = {}
        self.data = None
        self.device = device

    def load_data(self):
        d, self.header = read_dada_file(self.file_path, self.device)
        self.data = d.permute(2, 1, 0).cpu().numpy()  # (n_dat, n_chan, n_pol)
        return self

    @property
    def ndat(self):
        return 0 if self.data is None else self.data.shape[0]

    def __repr__(self):
        return f"DADAFile({self.file_path!r})"
