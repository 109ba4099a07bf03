"""Digest of the C2 round-trip output (development check: one-launch vs two-kernel paths
must agree bit for bit).  Prints one JSON line."""
import hashlib
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ska-pst-dsp-model_amd"), REPO]


def main():
    import torch
    import ska_pst_dsp_model_amd as pfb
    n_pol = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    os_ = sys.argv[2] if len(sys.argv) > 2 else "8/7"
    dev = torch.device("cuda", 0)
    taps = pfb.design_PFB_FIR_filter(256, os_, 12)
    n = 1 << 24
    g = torch.Generator(device=dev).manual_seed(100)
    x = (torch.complex(torch.randn((n_pol, n), device=dev, generator=g),
                       torch.randn((n_pol, n), device=dev, generator=g)) / np.sqrt(2)).to(torch.complex64)
    ana = pfb.AnalysisPlan(taps, 256, os_, "polyphase_analysis", n_pol, 0)
    win = pfb.PFBWindow().lookup["tukey"](256, 48)
    syn = pfb.SynthesisPlan(256, os_, 256, 48, True, 1, True, taps, win, None, n_pol, 0)
    res = {"env": {k: v for k, v in os.environ.items() if k.startswith("PFB_")}, "n_pol": n_pol, "os": os_}
    for it in range(3):
        chan, out = pfb.roundtrip(ana, syn, x)
        torch.cuda.synchronize()
        res[f"out_{it}"] = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
        res[f"chan_{it}"] = hashlib.sha256(chan.cpu().numpy().tobytes()).hexdigest()[:16]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
