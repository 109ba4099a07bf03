"""Digest of one round trip (channelised product and output) for A/B parity of kernel
variants: the same input, any library build (PFB_HIP_LIB), one JSON line with the SHA-256
of both buffers.  Variants that must be bit-identical print the same digests.

    PFB_HIP_LIB=ska-pst-dsp-model_amd/lib/libpfb_hip_exp.so PFB_W5_DEFER=0 \\
        python scripts/rt_digest.py --workload c3
"""
import argparse
import hashlib
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ska-pst-dsp-model_amd"), REPO]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=("c2", "c3"), default="c3")
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    import torch
    import ska_pst_dsp_model_amd as pfb
    dev = torch.device("cuda", 0)
    if args.workload == "c3":
        taps = pfb.design_PFB_FIR_filter_two_stage(4096, "8/7", 28)
        N, nf, ov, var, n = 4096, 512, 128, "polyphase_analysis_padded", 1 << 26
    else:
        taps = pfb.design_PFB_FIR_filter(256, "8/7", 12)
        N, nf, ov, var, n = 256, 256, 48, "polyphase_analysis", 1 << 24
    g = torch.Generator(device=dev).manual_seed(7)
    x = (torch.complex(torch.randn(n, device=dev, generator=g), torch.randn(n, device=dev, generator=g))
         / np.sqrt(2.0)).to(torch.complex64)[None]
    win = pfb.PFBWindow().lookup["tukey"](nf, ov)
    ana = pfb.AnalysisPlan(taps, N, "8/7", var, 1)
    syn = pfb.SynthesisPlan(N, "8/7", nf, ov, True, 1, True, taps, win, None, 1)
    chan, out = pfb.roundtrip(ana, syn, x)
    chan, out = pfb.roundtrip(ana, syn, x, chan=chan, out=out)  # second call: warm paths
    torch.cuda.synchronize()
    d = {"tag": args.tag, "workload": args.workload,
         "chan_sha": hashlib.sha256(chan.cpu().numpy().tobytes()).hexdigest()[:16],
         "out_sha": hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16],
         "pfb_env": {k: v for k, v in os.environ.items() if k.startswith("PFB_")}}
    print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
