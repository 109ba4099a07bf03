"""CPU tests of the C-ABI boundary: the library loads and exports every symbol that
include/pfb_api.h declares; without a GPU every plan call fails loudly."""
import ctypes
import os
import re

import pytest

from conftest import REPO


def _declared_symbols():
    with open(os.path.join(REPO, "include", "pfb_api.h")) as f:
        text = f.read()
    decl = r"^(?:pfb_status|int64_t|int32_t|double|const char\*)\s+(pfb_[a-z0-9_]+)\s*\("
    return sorted(set(re.findall(decl, text, flags=re.M)))


def test_header_symbols_are_exported():
    from ska_pst_dsp_model_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    declared = _declared_symbols()
    assert len(declared) >= 20
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing


def test_binding_covers_header():
    from ska_pst_dsp_model_amd import _lib
    bound = {name for name, _, _ in _lib.SYMBOLS}
    assert set(_declared_symbols()) == bound


def test_api_version_and_error_channel():
    from ska_pst_dsp_model_amd import _lib
    lib = _lib.load()
    assert lib.pfb_api_version() == 1
    st = lib.pfb_analysis_plan_create(None, None)
    assert st == _lib.PFB_ERR_INVALID_ARG
    assert b"null" in lib.pfb_last_error()


def test_struct_layouts_match_header():
    """ctypes mirrors of pfb_analysis_desc / pfb_synthesis_desc (x86-64 SysV ABI)."""
    from ska_pst_dsp_model_amd import _lib
    assert ctypes.sizeof(_lib.AnalysisDesc) == 40
    assert _lib.AnalysisDesc.taps.offset == 16 and _lib.AnalysisDesc.n_pol.offset == 32
    assert ctypes.sizeof(_lib.SynthesisDesc) == 88
    assert _lib.SynthesisDesc.taps.offset == 32
    assert _lib.SynthesisDesc.n_pol.offset == 80


def test_no_cpu_fallback_without_device():
    """The product path refuses to run without a HIP device (no silent fallback)."""
    import numpy as np
    import ska_pst_dsp_model_amd as pfb
    if pfb.device_count() > 0:
        pytest.skip("a GPU is present; this checks the CPU-only container")
    with pytest.raises(pfb.PfbError):
        pfb.polyphase_analysis(np.zeros((1, 1, 4096), np.complex64),
                               pfb.design_PFB_FIR_filter(8, "8/7", 10), 8, "8/7")
    with pytest.raises(pfb.PfbError):
        pfb.polyphase_synthesis(np.zeros((1, 8, 500), np.complex64), 1, 128, "8/7")


@pytest.mark.parametrize("args", [
    (5000, 8, "8/7", 81, 128, 16),           # 'test'
    (1 << 24, 256, "8/7", 3073, 256, 48),    # C2
    (1 << 26, 4096, "8/7", 100353, 512, 128),  # C3
    (1 << 20, 256, "4/3", 3073, 256, 48),    # 'low' 4/3
    (300000, 256, "32/27", 6145, 256, 54),   # normalize(os, Ov) non-integral (Matlab double)
    (100, 8, "8/7", 81, 128, 16),            # negative block counts (Matlab floor)
])
def test_calc_output_nbins_matches_oracle(args):
    """Product calc_output_nbins (C ABI, calc_output_nbins.m:17-27) == the oracle's."""
    import ska_pst_dsp_model_amd as pfb
    from oracle import pfb_oracle as orc
    nbins, ch, os_, taps, nf, ov = args
    got = pfb.calc_output_nbins(nbins, ch, os_, taps, nf, ov)
    ref = orc.calc_output_nbins(nbins, ch, os_, taps, nf, ov)
    assert float(got) == float(ref), (got, ref)
