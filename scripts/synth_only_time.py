"""Time the standalone C2 synthesis (SynthesisPlan.execute of an HBM-resident channelised
product — the PST production case, InverseFilterBank.m:92-96) with HIP events, for A/B of
library builds (PFB_HIP_LIB).  One JSON line.

    PFB_HIP_LIB=ska-pst-dsp-model_amd/lib/libpfb_hip_exp.so python scripts/synth_only_time.py
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ska-pst-dsp-model_amd"), REPO]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    import torch
    import ska_pst_dsp_model_amd as pfb
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(100)
    n = 1 << 24
    taps = pfb.design_PFB_FIR_filter(256, "8/7", 12)
    x = (torch.complex(torch.randn((1, n), device=dev, generator=g),
                       torch.randn((1, n), device=dev, generator=g)) / np.sqrt(2)).to(torch.complex64)
    ana = pfb.AnalysisPlan(taps, 256, "8/7", "polyphase_analysis", 1, 0)
    win = pfb.PFBWindow().lookup["tukey"](256, 48)
    syn = pfb.SynthesisPlan(256, "8/7", 256, 48, True, 1, True, taps, win, None, 1, 0)
    chan = ana.execute(x).contiguous()
    out = syn.execute(chan, layout="ptc")
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(args.reps):
        syn.execute(chan, layout="ptc")
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / args.reps
    print(json.dumps({"tag": args.tag, "workload": "C2 synthesis only", "ms": round(ms, 4),
                      "out_samples": int(out.shape[-1]),
                      "msamples_per_s": round(out.shape[-1] / ms / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
