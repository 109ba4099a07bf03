"""A few steps of one workload for rocprofv3 --pmc passes (scripts/gpu_pmc_r05.sh):
c2 = the fused C2 round trip (bench.py's step), c4 = the same for a dual-pol unit (bench.py
--gpus N > 1), c2syn / c4syn = the standalone synthesis (SynthesisPlan.execute of an
HBM-resident channelised product) of a single- / dual-pol unit (bench.py's synthesis_only at
--gpus 1 / > 1), c3 / c3p2 = the SKA-Mid round trip of a single- / dual-pol unit.
Every kernel name then maps to one workload in profiles/pmc_traffic.json."""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ska-pst-dsp-model_amd"), REPO]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=("c2", "c4", "c2syn", "c4syn", "c3", "c3p2"), required=True)
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    import torch
    import ska_pst_dsp_model_amd as pfb
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(100)
    if args.workload in ("c3", "c3p2"):
        taps = pfb.design_PFB_FIR_filter_two_stage(4096, "8/7", 28)
        N, nf, ov, var, n = 4096, 512, 128, "polyphase_analysis_padded", 1 << 26
    else:
        taps = pfb.design_PFB_FIR_filter(256, "8/7", 12)
        N, nf, ov, var, n = 256, 256, 48, "polyphase_analysis", 1 << 24
    n_pol = 2 if args.workload in ("c4", "c4syn", "c3p2") else 1
    x = (torch.complex(torch.randn((n_pol, n), device=dev, generator=g),
                       torch.randn((n_pol, n), device=dev, generator=g)) / np.sqrt(2)).to(torch.complex64)
    ana = pfb.AnalysisPlan(taps, N, "8/7", var, n_pol, 0)
    win = pfb.PFBWindow().lookup["tukey"](nf, ov)
    syn = pfb.SynthesisPlan(N, "8/7", nf, ov, True, 1, True, taps, win, None, n_pol, 0)
    if args.workload in ("c2syn", "c4syn"):
        chan = ana.execute(x).contiguous()
        torch.cuda.synchronize()
        for _ in range(args.steps):
            syn.execute(chan, layout="ptc")
    else:
        K = ana.output_length(n)
        chan = torch.empty((n_pol, K, N), dtype=torch.complex64, device=dev)
        out = torch.empty((n_pol, syn.output_length(K)), dtype=torch.complex64, device=dev)
        for _ in range(args.steps):
            pfb.roundtrip(ana, syn, x, chan=chan, out=out)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
