"""CPU tests of the C ABI's argument checking (include/pfb_api.h): every entry point
rejects null plans, bad sizes and inconsistent descriptors with a status and a message
(pfb_last_error), and the descriptor checks + host-side tables of plan creation run
without a device (pfb_*_plan_validate) for every BASELINE configuration.  These are the
host code paths tests/test_sanitize.py runs under AddressSanitizer + UBSan."""
import ctypes
from ctypes import POINTER, byref, c_double, c_int64, c_void_p

import numpy as np
import pytest


def _lib():
    from ska_pst_dsp_model_amd import _lib as L
    return L, L.load()


def _taps(n):
    t = np.hanning(n + 2)[1:-1].astype(np.float64)
    return t / t.sum()


def _ana_desc(L, variant=0, n_chan=256, nu=8, de=7, taps=None, n_pol=1, device=0):
    taps = _taps(3073) if taps is None else taps
    arr = np.ascontiguousarray(taps, dtype=np.float64)
    d = L.AnalysisDesc(variant, n_chan, nu, de, arr.ctypes.data_as(POINTER(c_double)) if len(arr) else None,
                       len(arr), n_pol, device)
    return d, arr


def _syn_desc(L, n_chan=256, nu=8, de=7, nf=256, ov=48, spans=1, combine=1, deripple=1, taps=None,
              tk=1, tco=None, sk=0, sco=None, n_pol=1, device=0):
    taps = _taps(3073) if taps is None else taps
    keep = [np.ascontiguousarray(taps, dtype=np.float64)]
    tp = keep[0].ctypes.data_as(POINTER(c_double)) if len(keep[0]) else None
    tcp = scp = None
    if tco is not None:
        keep.append(np.ascontiguousarray(tco, dtype=np.float64))
        tcp = keep[-1].ctypes.data_as(POINTER(c_double))
    if sco is not None:
        keep.append(np.ascontiguousarray(sco, dtype=np.float64))
        scp = keep[-1].ctypes.data_as(POINTER(c_double))
    d = L.SynthesisDesc(n_chan, nu, de, nf, ov, spans, combine, deripple, tp, len(keep[0]), tk, tcp, sk,
                        scp, n_pol, device)
    return d, keep


def _expect(lib, L, st, want):
    assert st == want, (st, want, lib.pfb_last_error())
    if want != L.PFB_OK:
        assert lib.pfb_last_error(), "an error status without a message"


# ---------------------------------------------------------------- descriptors
@pytest.mark.parametrize("variant,n_chan,nu,de,n_taps", [
    (0, 8, 8, 7, 81),          # C1 'test'
    (0, 256, 8, 7, 3073),      # C2 SKA-Low
    (0, 256, 4, 3, 3073),      # C2' reference 'low'
    (1, 4096, 8, 7, 100353),   # C3 SKA-Mid padded
    (1, 256, 8, 7, 3073),      # padded, streaming N
    (2, 256, 4, 3, 3072),      # LowCBF PST filterbank
    (0, 256, 32, 27, 6145),    # 'sps'-like ratio
    (0, 16, 8, 7, 161),        # two-stage stage 2 (16 ch)
])
def test_analysis_validate_accepts_baseline_configs(variant, n_chan, nu, de, n_taps):
    L, lib = _lib()
    d, _ = _ana_desc(L, variant, n_chan, nu, de, _taps(n_taps))
    _expect(lib, L, lib.pfb_analysis_plan_validate(byref(d)), L.PFB_OK)


@pytest.mark.parametrize("kw,status", [
    (dict(variant=7), "INVALID_ARG"),
    (dict(n_chan=0), "INVALID_ARG"),
    (dict(n_chan=-256), "INVALID_ARG"),
    (dict(nu=7, de=8), "INVALID_ARG"),            # os_de > os_nu
    (dict(nu=0), "INVALID_ARG"),
    (dict(taps=np.zeros(0)), "INVALID_ARG"),
    (dict(n_pol=0), "INVALID_ARG"),
    (dict(n_pol=70000), "INVALID_ARG"),
    (dict(variant=2, n_chan=256, nu=8, de=7), "INVALID_ARG"),  # LowCBF is fixed 256 ch 4/3 3072 taps
    (dict(n_chan=1 << 30), "UNSUPPORTED"),
    (dict(n_chan=1, nu=8, de=7), "INVALID_ARG"),  # M = floor(1 * 7 / 8) = 0
    (dict(n_chan=48), "UNSUPPORTED"),             # no kernel for a non-power-of-two N
])
def test_analysis_validate_rejects(kw, status):
    L, lib = _lib()
    d, _ = _ana_desc(L, **kw)
    _expect(lib, L, lib.pfb_analysis_plan_validate(byref(d)), getattr(L, "PFB_ERR_" + status))
    # plan creation reports the same status before it looks for a device
    h = c_void_p()
    _expect(lib, L, lib.pfb_analysis_plan_create(byref(d), byref(h)), getattr(L, "PFB_ERR_" + status))
    assert not h.value


@pytest.mark.parametrize("kw", [
    dict(),                                                   # C2
    dict(nu=4, de=3),                                         # C2'
    dict(n_chan=4096, nf=512, ov=128, taps=_taps(100353)),    # C3
    dict(n_chan=4096, nf=256, ov=32, taps=_taps(100353)),     # mid_external
    dict(n_chan=8, nf=128, ov=16, taps=_taps(81)),            # C1 'test'
    dict(spans=0, deripple=0),                                # critical
    dict(combine=4),                                          # combine permutation
    dict(tk=3),                                               # hann temporal quirk (per channel)
    dict(tk=2),                                               # top_hat
    dict(tk=0),                                               # no_window
    dict(tk=4, tco=np.linspace(0.5, 1.0, 256)),               # custom temporal
    dict(sk=3),                                               # hann spectral taper
    dict(sk=4, sco=np.ones(256 * 224)),                       # custom spectral (L values)
    dict(n_chan=8, nu=32, de=27, nf=256, ov=64, taps=_taps(81), deripple=0),  # 'sps'-like
    dict(n_chan=8, nu=32, de=27, nf=256, ov=48, taps=_taps(81), deripple=0),  # L_ov = 40.5 N
])
def test_synthesis_validate_accepts(kw):
    L, lib = _lib()
    d, _keep = _syn_desc(L, **kw)
    _expect(lib, L, lib.pfb_synthesis_plan_validate(byref(d)), L.PFB_OK)


@pytest.mark.parametrize("kw,status", [
    (dict(n_chan=0), "INVALID_ARG"),
    (dict(nf=250), "INVALID_ARG"),                   # Nf de / nu not integral
    (dict(ov=47), "INVALID_ARG"),                    # Ov de N / nu not integral (8 ch, 32/27)
    (dict(ov=128), "INVALID_ARG"),                   # keep = Nf - 2 Ov <= 0
    (dict(ov=(1 << 31) - 1), "INVALID_ARG"),         # overflow-safe keep check
    (dict(nf=(1 << 31) - 1), "UNSUPPORTED"),         # beyond the 32-bit table sizes
    (dict(combine=3), "INVALID_ARG"),                # combine must divide n_chan
    (dict(combine=0), "INVALID_ARG"),
    (dict(sk=1), "INVALID_ARG"),                     # tukey as a spectral taper
    (dict(sk=4), "INVALID_ARG"),                     # custom spectral without coefficients
    (dict(tk=4), "INVALID_ARG"),                     # custom temporal without coefficients
    (dict(tk=9), "INVALID_ARG"),                     # unknown temporal taper
    (dict(deripple=1, taps=np.zeros(0)), "INVALID_ARG"),
    (dict(n_pol=0), "INVALID_ARG"),
    (dict(n_pol=1 << 17), "INVALID_ARG"),
    (dict(nf=96, ov=16, nu=4, de=3), "UNSUPPORTED"),  # no synthesis kernel for Nf 96
])
def test_synthesis_validate_rejects(kw, status):
    L, lib = _lib()
    if kw.get("ov") == 47:  # 47 * 27 * 8 / 32 = 317.25
        kw = dict(kw, n_chan=8, nu=32, de=27, taps=_taps(81), nf=256)
    d, _keep = _syn_desc(L, **kw)
    want = getattr(L, "PFB_ERR_" + status)
    _expect(lib, L, lib.pfb_synthesis_plan_validate(byref(d)), want)
    h = c_void_p()
    _expect(lib, L, lib.pfb_synthesis_plan_create(byref(d), byref(h)), want)
    assert not h.value


def test_null_descriptors():
    L, lib = _lib()
    h = c_void_p()
    _expect(lib, L, lib.pfb_analysis_plan_validate(None), L.PFB_ERR_INVALID_ARG)
    _expect(lib, L, lib.pfb_synthesis_plan_validate(None), L.PFB_ERR_INVALID_ARG)
    _expect(lib, L, lib.pfb_analysis_plan_create(None, byref(h)), L.PFB_ERR_INVALID_ARG)
    _expect(lib, L, lib.pfb_synthesis_plan_create(None, byref(h)), L.PFB_ERR_INVALID_ARG)
    d, _ = _ana_desc(L)
    _expect(lib, L, lib.pfb_analysis_plan_create(byref(d), None), L.PFB_ERR_INVALID_ARG)


# ---------------------------------------------------------------- null plans
def test_null_plan_calls_fail_cleanly():
    L, lib = _lib()
    n = c_int64(0)
    buf = (ctypes.c_float * 64)()
    p = ctypes.cast(buf, c_void_p)
    E = L.PFB_ERR_INVALID_ARG
    _expect(lib, L, lib.pfb_analysis_execute(None, p, 8, 8, p, 8, 8, byref(n), 0, None), E)
    _expect(lib, L, lib.pfb_filterbank_execute(None, p, 8, 8, p, 8, 8, byref(n), 0, None), E)
    _expect(lib, L, lib.pfb_filterbank_execute_strided(None, p, 8, 8, p, 8, 1, 1, 0, 0, 0, 8,
                                                        byref(n), None), E)
    _expect(lib, L, lib.pfb_filterbank_reset(None), E)
    _expect(lib, L, lib.pfb_synthesis_execute(None, p, 8, 8, 1, p, 8, 8, byref(n), 0, None), E)
    _expect(lib, L, lib.pfb_inverse_filterbank_execute(None, p, 8, 8, p, 8, 8, byref(n), 0, None), E)
    _expect(lib, L, lib.pfb_inverse_filterbank_reset(None), E)
    _expect(lib, L, lib.pfb_inverse_filterbank_set_sample_offset(None, 3), E)
    _expect(lib, L, lib.pfb_synthesis_set_chunk_blocks(None, 4), E)
    _expect(lib, L, lib.pfb_synthesis_set_stage1_rows(None, 1), E)
    _expect(lib, L, lib.pfb_roundtrip_execute(None, None, p, 8, 8, p, 8, 8, byref(n), 1, p, 8, 8,
                                              byref(n), None), E)
    _expect(lib, L, lib.pfb_roundtrip_analysis_execute(None, None, p, 8, 8, p, 8, 8, byref(n), 1, None), E)
    _expect(lib, L, lib.pfb_roundtrip_synthesis_execute(None, None, 8, 1, p, 8, 8, byref(n), None), E)
    assert lib.pfb_analysis_output_length(None, 100) == -1
    assert lib.pfb_analysis_output_channels(None) == -1
    assert lib.pfb_filterbank_buffered(None) == -1
    assert lib.pfb_filterbank_output_rows(None, 10) == -1
    assert lib.pfb_synthesis_output_length(None, 100) == -1
    assert lib.pfb_inverse_filterbank_buffered(None) == -1
    assert lib.pfb_synthesis_last_stage1_rows(None) == -1
    # destroying nothing is a no-op
    assert lib.pfb_analysis_plan_destroy(None) == L.PFB_OK
    assert lib.pfb_synthesis_plan_destroy(None) == L.PFB_OK


# ---------------------------------------------------------------- layout / utilities
def test_layout_entry_points_reject_bad_arguments():
    L, lib = _lib()
    E = L.PFB_ERR_INVALID_ARG
    buf = (ctypes.c_float * 256)()
    p = ctypes.cast(buf, c_void_p)
    _expect(lib, L, lib.pfb_dada_unpack(p, 8, 2, 0, -1, 1, 1, p, 8, None), E)      # negative n_dat
    _expect(lib, L, lib.pfb_dada_unpack(p, 8, 3, 0, 8, 1, 1, p, 8, None), E)       # NDIM 3
    _expect(lib, L, lib.pfb_dada_unpack(p, 8, 2, 5, 8, 1, 1, p, 8, None), E)       # unknown order
    _expect(lib, L, lib.pfb_dada_unpack(p, 8, 2, 1, 33, 1, 1, p, 64, None), E)     # LowCBF heap of 32
    _expect(lib, L, lib.pfb_dada_unpack(p, 8, 2, 0, 8, 2, 1, p, 8, None), E)       # stride too small
    _expect(lib, L, lib.pfb_dada_unpack(None, 8, 2, 0, 8, 1, 1, p, 8, None), E)    # null input
    assert lib.pfb_dada_unpack(None, 8, 2, 0, 0, 1, 1, None, 0, None) == L.PFB_OK  # nothing to do
    _expect(lib, L, lib.pfb_dada_pack(p, 8, 8, 0, 1, p, 8, None), E)               # n_chan 0
    _expect(lib, L, lib.pfb_dada_pack(p, 4, 8, 1, 1, p, 8, None), E)               # stride too small
    _expect(lib, L, lib.pfb_dada_pack(None, 8, 8, 1, 1, p, 8, None), E)
    _expect(lib, L, lib.pfb_gather_channels(p, 8, 8, p, 8, 8, -1, 1, 1, 0, 0, 0, None), E)
    _expect(lib, L, lib.pfb_gather_channels(p, 8, 8, p, 8, 8, 70000, 1, 1, 0, 0, 0, None), E)
    _expect(lib, L, lib.pfb_gather_channels(p, 8, 8, p, 8, 8, 1, 2, 4, 6, 8, 0, None), E)  # past the row
    _expect(lib, L, lib.pfb_gather_channels(None, 8, 8, p, 8, 8, 1, 1, 1, 0, 0, 0, None), E)
    _expect(lib, L, lib.pfb_corner_turn(p, 8, 8, -1, 8, 8, p, 8, 8, None), E)
    _expect(lib, L, lib.pfb_corner_turn(p, 8, 8, 70000, 8, 8, p, 8, 8, None), E)
    _expect(lib, L, lib.pfb_corner_turn(None, 8, 8, 1, 8, 8, p, 8, 8, None), E)
    sc = c_double(0.0)
    _expect(lib, L, lib.pfb_quantize(p, 8, -1, 1, 1.0, p, 8, byref(sc), None), E)
    _expect(lib, L, lib.pfb_quantize(p, 4, 8, 1, 1.0, p, 8, byref(sc), None), E)
    _expect(lib, L, lib.pfb_quantize(None, 8, 8, 1, 1.0, p, 8, byref(sc), None), E)
    _expect(lib, L, lib.pfb_quantize(p, 1, 1, 1, 1.0, p, 1, byref(sc), None), E)  # var of one sample
    _expect(lib, L, lib.pfb_device_copy(p, p, 63, None), E)                          # not a multiple of 64
    _expect(lib, L, lib.pfb_device_copy(None, p, 64, None), E)
    _expect(lib, L, lib.pfb_device_malloc(0, -1, None), E)


def test_profile_and_query_arguments():
    L, lib = _lib()
    E = L.PFB_ERR_INVALID_ARG
    ms, nl, by = c_double(), c_int64(), c_double()
    for w in range(6):
        assert lib.pfb_profile_read(w, byref(ms), byref(nl), byref(by)) == L.PFB_OK
    _expect(lib, L, lib.pfb_profile_read(6, byref(ms), byref(nl), byref(by)), E)
    _expect(lib, L, lib.pfb_profile_read(-1, None, None, None), E)
    buf = ctypes.create_string_buffer(8)
    _expect(lib, L, lib.pfb_profile_kernel_name(0, None, 8), E)
    _expect(lib, L, lib.pfb_profile_kernel_name(0, buf, 0), E)
    _expect(lib, L, lib.pfb_profile_kernel_name(9, buf, 8), E)
    assert lib.pfb_profile_kernel_name(0, buf, 1) == L.PFB_OK and buf.value == b""
    assert lib.pfb_profile_reset() == L.PFB_OK


@pytest.mark.parametrize("args", [
    (0, 1, 1, 1, 0, 2, 0),
    ((1 << 62), 4096, 8, 7, 100353, 512, 128),
    (-(1 << 40), 256, 8, 7, 3073, 256, 48),
    (1 << 26, 65536, 1 << 15, 1, 1, 1 << 20, 1 << 18),
])
def test_calc_output_nbins_extremes_are_finite(args):
    """calc_output_nbins.m:17-27 in double arithmetic: finite for extreme arguments (a UBSan
    target: no integer arithmetic on them)."""
    L, lib = _lib()
    v = lib.pfb_calc_output_nbins(*args)
    assert np.isfinite(v)
