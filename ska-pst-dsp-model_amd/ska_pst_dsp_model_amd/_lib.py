"""ctypes binding of the C ABI declared in ``include/pfb_api.h``.

The shared library ``libpfb_hip.so`` is built in-tree (``ska-pst-dsp-model_amd/lib``)
by ``__graft_entry__.build()`` / ``make -C ska-pst-dsp-model_amd``.  There is no CPU
fallback: if the library cannot be loaded, or no HIP device is present, every product
call raises ``PfbError``.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, Structure, c_char_p, c_double, c_float, c_int32, c_int64,
                    c_void_p)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.normpath(os.path.join(_HERE, "..", "lib"))
LIB_PATH = os.environ.get("PFB_HIP_LIB", os.path.join(LIB_DIR, "libpfb_hip.so"))

PFB_OK = 0
PFB_ERR_INVALID_ARG = 1
PFB_ERR_UNSUPPORTED = 2
PFB_ERR_HIP = 3
PFB_ERR_OOM = 4
PFB_ERR_BUFFER_TOO_SMALL = 5
PFB_ERR_NO_DEVICE = 6

PFB_ANALYSIS_BUNTON = 0
PFB_ANALYSIS_PADDED = 1
PFB_ANALYSIS_LOWCBF = 2
PFB_MEM_DEVICE = 0
PFB_MEM_HOST = 1

PFB_WINDOW_NONE = 0
PFB_WINDOW_TUKEY = 1
PFB_WINDOW_TOP_HAT = 2
PFB_WINDOW_HANN = 3
PFB_WINDOW_CUSTOM = 4

PFB_STAGE1_AUTO = 0
PFB_STAGE1_STORED = 1
PFB_STAGE1_RECOMPUTED = 2
PFB_DADA_TFP = 0
PFB_DADA_LOWCBF = 1

_STATUS_NAMES = {
    0: "PFB_OK", 1: "PFB_ERR_INVALID_ARG", 2: "PFB_ERR_UNSUPPORTED", 3: "PFB_ERR_HIP",
    4: "PFB_ERR_OOM", 5: "PFB_ERR_BUFFER_TOO_SMALL", 6: "PFB_ERR_NO_DEVICE",
}


class PfbError(RuntimeError):
    """Raised for any non-OK status of the C ABI (mirrors the reference's error(...))."""

    def __init__(self, status: int, message: str):
        self.status = status
        super().__init__(f"{_STATUS_NAMES.get(status, status)}: {message}")


class AnalysisDesc(Structure):
    _fields_ = [("variant", c_int32), ("n_chan", c_int32), ("os_nu", c_int32),
                ("os_de", c_int32), ("taps", POINTER(c_double)), ("n_taps", c_int64),
                ("n_pol", c_int32), ("device", c_int32)]


class SynthesisDesc(Structure):
    _fields_ = [("n_chan", c_int32), ("os_nu", c_int32), ("os_de", c_int32),
                ("input_fft_length", c_int32), ("input_overlap", c_int32),
                ("spans_nyquist", c_int32), ("combine", c_int32),
                ("apply_deripple", c_int32), ("taps", POINTER(c_double)), ("n_taps", c_int64),
                ("temporal_taper", c_int32), ("temporal_coeffs", POINTER(c_double)),
                ("spectral_taper", c_int32), ("spectral_coeffs", POINTER(c_double)),
                ("n_pol", c_int32), ("device", c_int32)]


# (name, restype, argtypes) of every exported symbol in include/pfb_api.h
SYMBOLS = [
    ("pfb_analysis_plan_create", c_int32, [POINTER(AnalysisDesc), POINTER(c_void_p)]),
    ("pfb_analysis_plan_destroy", c_int32, [c_void_p]),
    ("pfb_analysis_plan_validate", c_int32, [POINTER(AnalysisDesc)]),
    ("pfb_analysis_output_length", c_int64, [c_void_p, c_int64]),
    ("pfb_analysis_output_channels", c_int32, [c_void_p]),
    ("pfb_analysis_execute", c_int32, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_int64,
                                       c_int64, POINTER(c_int64), c_int32, c_void_p]),
    ("pfb_filterbank_execute", c_int32, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_int64,
                                         c_int64, POINTER(c_int64), c_int32, c_void_p]),
    ("pfb_filterbank_buffered", c_int64, [c_void_p]),
    ("pfb_filterbank_reset", c_int32, [c_void_p]),
    ("pfb_filterbank_output_rows", c_int64, [c_void_p, c_int64]),
    ("pfb_filterbank_execute_strided", c_int32, [c_void_p, c_void_p, c_int64, c_int64, c_void_p,
                                                 c_int64, c_int64, c_int64, c_int32, c_int32,
                                                 c_int32, c_int64, POINTER(c_int64), c_void_p]),
    ("pfb_synthesis_plan_create", c_int32, [POINTER(SynthesisDesc), POINTER(c_void_p)]),
    ("pfb_synthesis_plan_destroy", c_int32, [c_void_p]),
    ("pfb_synthesis_plan_validate", c_int32, [POINTER(SynthesisDesc)]),
    ("pfb_synthesis_output_length", c_int64, [c_void_p, c_int64]),
    ("pfb_synthesis_execute", c_int32, [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_void_p,
                                        c_int64, c_int64, POINTER(c_int64), c_int32, c_void_p]),
    ("pfb_inverse_filterbank_execute", c_int32, [c_void_p, c_void_p, c_int64, c_int64, c_void_p,
                                                 c_int64, c_int64, POINTER(c_int64), c_int32,
                                                 c_void_p]),
    ("pfb_inverse_filterbank_buffered", c_int64, [c_void_p]),
    ("pfb_inverse_filterbank_reset", c_int32, [c_void_p]),
    ("pfb_inverse_filterbank_set_sample_offset", c_int32, [c_void_p, c_int64]),
    ("pfb_synthesis_set_chunk_blocks", c_int32, [c_void_p, c_int32]),
    ("pfb_synthesis_set_stage1_rows", c_int32, [c_void_p, c_int32]),
    ("pfb_synthesis_last_stage1_rows", c_int32, [c_void_p]),
    ("pfb_roundtrip_execute", c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_int64,
                                        c_void_p, c_int64, c_int64, POINTER(c_int64), c_int64,
                                        c_void_p, c_int64, c_int64, POINTER(c_int64), c_void_p]),
    ("pfb_roundtrip_analysis_execute", c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_int64,
                                                 c_void_p, c_int64, c_int64, POINTER(c_int64),
                                                 c_int64, c_void_p]),
    ("pfb_roundtrip_synthesis_execute", c_int32, [c_void_p, c_void_p, c_int64, c_int64, c_void_p,
                                                  c_int64, c_int64, POINTER(c_int64), c_void_p]),
    ("pfb_dada_unpack", c_int32, [c_void_p, c_int32, c_int32, c_int32, c_int64, c_int32,
                                  c_int32, c_void_p, c_int64, c_void_p]),
    ("pfb_dada_pack", c_int32, [c_void_p, c_int64, c_int64, c_int32, c_int32, c_void_p, c_int32,
                                c_void_p]),
    ("pfb_gather_channels", c_int32, [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int64,
                                      c_int64, c_int64, c_int32, c_int32, c_int32, c_int32,
                                      c_void_p]),
    ("pfb_corner_turn", c_int32, [c_void_p, c_int64, c_int64, c_int64, c_int64, c_int64,
                                  c_void_p, c_int64, c_int64, c_void_p]),
    ("pfb_quantize", c_int32, [c_void_p, c_int64, c_int64, c_int32, c_double, c_void_p, c_int64,
                               POINTER(c_double), c_void_p]),
    ("pfb_calc_output_nbins", c_double, [c_int64, c_int32, c_int32, c_int32, c_int64, c_int32,
                                         c_int32]),
    ("pfb_last_error", c_char_p, []),
    ("pfb_api_version", c_int32, []),
    ("pfb_device_count", c_int32, []),
    ("pfb_device_malloc", c_int32, [c_int32, c_int64, POINTER(c_void_p)]),
    ("pfb_device_free", c_int32, [c_void_p]),
    ("pfb_memcpy_h2d", c_int32, [c_void_p, c_void_p, c_int64, c_void_p]),
    ("pfb_memcpy_d2h", c_int32, [c_void_p, c_void_p, c_int64, c_void_p]),
    ("pfb_stream_synchronize", c_int32, [c_void_p]),
    ("pfb_device_copy", c_int32, [c_void_p, c_void_p, c_int64, c_void_p]),
    ("pfb_profile_enable", c_int32, [c_int32]),
    ("pfb_profile_read", c_int32, [c_int32, POINTER(c_double), POINTER(c_int64),
                                   POINTER(c_double)]),
    ("pfb_profile_reset", c_int32, []),
    ("pfb_profile_kernel_name", c_int32, [c_int32, c_char_p, c_int64]),
    ("pfb_build_flags", c_int32, []),
]

_lib = None


def load(path: str = None):
    """Load (once) and return the ctypes library handle; raises PfbError if absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise PfbError(PFB_ERR_NO_DEVICE,
                       f"HIP extension not built: {p} is missing "
                       "(run __graft_entry__.build() or make -C ska-pst-dsp-model_amd)")
    lib = ctypes.CDLL(p)
    for name, res, args in SYMBOLS:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def check(status: int):
    if status != PFB_OK:
        msg = load().pfb_last_error()
        raise PfbError(status, msg.decode() if msg else "")


def device_count() -> int:
    return int(load().pfb_device_count())


def require_device():
    if device_count() <= 0:
        raise PfbError(PFB_ERR_NO_DEVICE,
                       "no HIP device: the PFB engine has no CPU fallback by design")


def c_double_array(values):
    import numpy as np
    arr = np.ascontiguousarray(values, dtype=np.float64)
    return arr, arr.ctypes.data_as(POINTER(c_double))
