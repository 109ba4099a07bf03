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

# The reference's parity criterion: np.isclose(a, b, atol=1e-6, rtol=1e-6) on raw
# unit-amplitude round-trip data (python/verify/test_matlab_dspsr_pfb_inversion.py:35,151).
# assert_pfb_close applies it literally:
#   * scale=1.0 — raw values (round trips of unit-amplitude inputs: the reference's case);
#   * scale="rms" (default) — both sides divided by the oracle's RMS magnitude, i.e. the
#     data brought to unit amplitude first (channelised products carry the analysis gain
#     N * |h|, synthesis-only inputs the inverse);
#   * scale="peak" — divided by the oracle's peak (|peak| ~ 4-5 x RMS on noise, so ~5x
#     looser; kept only for closed-form known answers whose values span decades).
# Every call reports max and RMS error relative to the same scale; with PFB_PARITY_LOG
# set, the numbers are appended there as JSON lines (profiles/r02_parity_errors.jsonl).
PARITY_TOL = 1e-6


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the HIP extension")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def parity_stats(got, ref, scale="rms"):
    """(scale used, max |got-ref| / scale, rms |got-ref| / scale, isclose fraction)."""
    got = np.asarray(got)
    ref = np.asarray(ref)
    if isinstance(scale, str):
        a = np.abs(ref.astype(np.complex128))
        s = float(np.sqrt(np.mean(a * a))) if scale == "rms" else float(a.max()) if a.size else 1.0
    else:
        s = float(scale)
    s = s if s > 0 else 1.0
    if not got.size:
        return s, 0.0, 0.0, 1.0
    d = np.abs(got.astype(np.complex128) - ref.astype(np.complex128)) / s
    return s, float(d.max()), float(np.sqrt(np.mean(d * d))), None


def assert_pfb_close(got, ref, tol=PARITY_TOL, scale="rms", what=""):
    got = np.asarray(got)
    ref = np.asarray(ref)
    assert got.shape == ref.shape, f"{what}: shape {got.shape} != {ref.shape}"
    s, emax, erms, _ = parity_stats(got, ref, scale)
    ok = np.isclose(got / s, ref / s, atol=tol, rtol=tol) if got.size else np.ones(1, bool)
    frac = float(ok.mean())
    # isclose margin: max |got - ref| / (atol + rtol |ref|) on the scaled values (np.isclose
    # passes a sample at <= 1; the margin says how close the worst sample came)
    if got.size:
        g = got.astype(np.complex128) / s
        r = ref.astype(np.complex128) / s
        margin = float((np.abs(g - r) / (tol + tol * np.abs(r))).max())
    else:
        margin = 0.0
    log = os.environ.get("PFB_PARITY_LOG")
    if log:
        import json
        test = os.environ.get("PYTEST_CURRENT_TEST", "").split(" ")[0]
        with open(log, "a") as f:
            f.write(json.dumps({"test": test, "what": what, "n": int(got.size),
                                "scale": scale if isinstance(scale, str) else "raw",
                                "scale_value": s, "tol": tol, "max_err": emax, "rms_err": erms,
                                "isclose_frac": frac, "margin": margin}) + "\n")
    assert frac == 1.0, (f"{what}: isclose({tol}) fraction {frac:.6f}; error / {scale} scale: "
                         f"max {emax:.3e}, rms {erms:.3e}, margin {margin:.3f}")
    return emax


@pytest.fixture(scope="session")
def gpu():
    """Skip-free GPU fixture: tests marked gpu must fail loudly without a device."""
    import torch
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    import ska_pst_dsp_model_amd as pfb
    assert pfb.device_count() > 0
    return torch.device("cuda:0")
