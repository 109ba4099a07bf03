"""Golden vectors of the reference's purity metrics (python/verify/util.py:15-43).

Run in the build container only (it reads /root/reference, which never travels to the GPU
box): imports the reference module from its file and writes its outputs on fixed arrays to
verify_util_golden.npz (arrays only, no pickles).  tests/test_formats_cpu.py compares
ska_pst_dsp_model_amd.verify with the file.

    python tests/golden/make_verify_util_golden.py
"""
import importlib.util
import os

import numpy as np

REF = "/root/reference/python/verify/util.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "verify_util_golden.npz")


def main():
    import matplotlib
    matplotlib.use("Agg")  # util.py imports pyplot at module level
    spec = importlib.util.spec_from_file_location("ref_verify_util", REF)
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)
    rng = np.random.default_rng(20261017)
    cases = {
        # noise with one dominant bin (a tone) — the TestPureTone shape
        "tone": np.concatenate([1e-4 * (rng.standard_normal(255) + 1j * rng.standard_normal(255)),
                                [3.0 + 4.0j]]),
        # an impulse response: peak at 0 dB, a few sidelobes
        "impulse": np.r_[np.zeros(40), 1e-3, -2e-3j, 1.0, 5e-4, np.zeros(60)].astype(np.complex128),
        # real noise, and a tie for the maximum (argmax takes the first)
        "noise": rng.standard_normal(1000),
        "tie": np.array([0.5, 2.0, 1.0, 2.0, -2.0]),
        # float32 data as the device returns it
        "single": (rng.standard_normal(4096) + 1j * rng.standard_normal(4096)).astype(np.complex64),
        "zeros": np.zeros(16),
    }
    out = {}
    for name, a in cases.items():
        out[f"{name}__in"] = a
        out[f"{name}__spurious"] = ref.spurious(np.abs(a) ** 2)
        out[f"{name}__total_spurious"] = np.asarray(ref.total_spurious(a))
        out[f"{name}__mean_spurious"] = np.asarray(ref.mean_spurious(a))
        out[f"{name}__max_spurious"] = np.asarray(ref.max_spurious(a))
        out[f"{name}__dB"] = ref.dB(np.abs(a) ** 2)
    np.savez(OUT, **out)
    print(f"wrote {OUT}: {len(cases)} cases")


if __name__ == "__main__":
    main()
