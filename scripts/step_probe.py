"""Step-time probe (development tool, experiments build): microseconds per C2 round-trip
step (2^24 samples, one unit) with plain stream launches and with one HIP graph per step,
as bench.py times it.  Variants are separate processes with PFB_* knobs set (the
experiments build reads them).  One JSON line: median over --reps timings of --steps steps.
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
    ap.add_argument("--tag", default="")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--n-pol", type=int, default=1)
    args = ap.parse_args()
    import torch
    import ska_pst_dsp_model_amd as pfb
    dev = torch.device("cuda", 0)
    taps = pfb.design_PFB_FIR_filter(256, "8/7", 12)
    n = 1 << 24
    g = torch.Generator(device=dev).manual_seed(100)
    x = (torch.complex(torch.randn((args.n_pol, n), device=dev, generator=g),
                       torch.randn((args.n_pol, n), device=dev, generator=g)) / np.sqrt(2)).to(torch.complex64)
    ana = pfb.AnalysisPlan(taps, 256, "8/7", "polyphase_analysis", args.n_pol, 0)
    win = pfb.PFBWindow().lookup["tukey"](256, 48)
    syn = pfb.SynthesisPlan(256, "8/7", 256, 48, True, 1, True, taps, win, None, args.n_pol, 0)
    K = ana.output_length(n)
    chan = torch.empty((args.n_pol, K, 256), dtype=torch.complex64, device=dev)
    out = torch.empty((args.n_pol, syn.output_length(K)), dtype=torch.complex64, device=dev)

    def step():
        pfb.roundtrip(ana, syn, x, chan=chan, out=out)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    ref = out.clone()
    graph = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream(device=dev)
    cs.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(cs):
        step()
    torch.cuda.current_stream(dev).wait_stream(cs)
    with torch.cuda.graph(graph):
        step()
    torch.cuda.synchronize()

    def timed(fn):
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(args.steps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / args.steps)
        return round(float(np.median(ts)), 1)

    res = {"tag": args.tag, "env": {k: v for k, v in os.environ.items() if k.startswith("PFB_") and k != "PFB_HIP_LIB"}}
    res["plain_us"] = timed(step)
    res["graph_us"] = timed(graph.replay)
    res["plain_us_2"] = timed(step)
    res["graph_us_2"] = timed(graph.replay)
    torch.cuda.synchronize()
    res["same_output"] = bool(torch.equal(out, ref))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
