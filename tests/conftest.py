"""Shared pytest configuration: the ``gpu`` marker, import paths and tolerances."""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "ska-pst-dsp-model_amd")
for p in (PKG_ROOT, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")

# The reference's parity criterion: np.isclose(a, b, atol=1e-6, rtol=1e-6) on
# unit-amplitude round-trip data (python/verify/test_matlab_dspsr_pfb_inversion.py:35,151).
# Channelised data are compared after dividing both sides by the oracle's peak
# magnitude, so the same 1e-6 applies at every stage.
PARITY_TOL = 1e-6


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the HIP extension")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def assert_pfb_close(got, ref, tol=PARITY_TOL, scale=None, what=""):
    got = np.asarray(got)
    ref = np.asarray(ref)
    assert got.shape == ref.shape, f"{what}: shape {got.shape} != {ref.shape}"
    s = float(np.abs(ref).max()) if scale is None else float(scale)
    s = s if s > 0 else 1.0
    ok = np.isclose(got / s, ref / s, atol=tol, rtol=tol)
    frac = ok.mean() if ok.size else 1.0
    err = np.abs(got - ref).max() / s if ok.size else 0.0
    assert frac == 1.0, f"{what}: isclose fraction {frac:.6f}, max rel-to-peak err {err:.3e}"
    return err


@pytest.fixture(scope="session")
def gpu():
    """Skip-free GPU fixture: tests marked gpu must fail loudly without a device."""
    import torch
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    import ska_pst_dsp_model_amd as pfb
    assert pfb.device_count() > 0
    return torch.device("cuda:0")
