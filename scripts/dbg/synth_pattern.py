"""Debug: where does the GPU synthesis differ from the oracle (pol / sample parity / block)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "ska-pst-dsp-model_amd"), REPO, os.path.join(REPO, "tests")]
import torch
import ska_pst_dsp_model_amd as pfb
from oracle import pfb_oracle as orc



import tests.test_gpu_parity as T
taps = T._taps("test")
rng = np.random.default_rng(21)
for (npol, N, nf, ov) in [(2, 8, 128, 16), (1, 8, 128, 16), (1, 256, 256, 48)]:
    x = T._noise(rng, (npol, N, 96 * 7 + 32 + 5)) if N == 8 else T._noise(rng, (npol, N, 160 * 4 + 96))
    t = taps if N == 8 else pfb.design_PFB_FIR_filter(256, "8/7", 12)
    got, ref = T._synth_case(pfb, x, 1, nf, "8/7", 1, t, ov, "tukey")
    s = np.abs(ref).max()
    bad = ~np.isclose(got / s, ref / s, atol=1e-6, rtol=1e-6)
    print(f"npol={npol} N={N} shape={ref.shape} bad frac={bad.mean():.4f}")
    if bad.any():
        idx = np.argwhere(bad)
        print("  first bad idx", idx[:8].tolist())
        b = bad.reshape(-1, bad.shape[-1]) if bad.ndim > 1 else bad
        print("  bad per pol", [float(bad[p].mean()) for p in range(bad.shape[0])])
        flat = bad.reshape(bad.shape[0], -1)
        print("  even/odd sample bad", float(flat[:, 0::2].mean()), float(flat[:, 1::2].mean()))
        g = got.reshape(-1); r = ref.reshape(-1)
        print("  got", g[:6], "\n  ref", r[:6])
