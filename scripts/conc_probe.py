"""Concurrency probe (development tool, experiments build): do the two C2 round-trip kernels
overlap when two independent units run on two streams?

Two independent (analysis, synthesis) plan pairs on 2^24-sample units.  Modes:
  serial  both units' round trips one after the other on one stream
  conc    unit 0 on stream 0, unit 1 on stream 1 (the GPU may overlap unit 1's analysis with
          unit 0's synthesis)
Prints one JSON line per mode: microseconds per unit round trip (median of --reps timings
of --iters iterations).  Grid sizes come from the experiments knobs PFB_ANA_WG_PER_CU and
PFB_WAVE_PER_CU.
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
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    import ska_pst_dsp_model_amd as pfb
    dev = torch.device("cuda", 0)
    taps = pfb.design_PFB_FIR_filter(256, "8/7", 12)
    n = 1 << 24
    units = []
    for u in range(2):
        g = torch.Generator(device=dev).manual_seed(100 + u)
        x = (torch.complex(torch.randn((1, n), device=dev, generator=g),
                           torch.randn((1, n), device=dev, generator=g)) / np.sqrt(2)).to(torch.complex64)
        ana = pfb.AnalysisPlan(taps, 256, "8/7", "polyphase_analysis", 1, 0)
        win = pfb.PFBWindow().lookup["tukey"](256, 48)
        syn = pfb.SynthesisPlan(256, "8/7", 256, 48, True, 1, True, taps, win, None, 1, 0)
        K = ana.output_length(n)
        chan = torch.empty((1, K, 256), dtype=torch.complex64, device=dev)
        out = torch.empty((1, syn.output_length(K)), dtype=torch.complex64, device=dev)
        units.append((ana, syn, x, chan, out))
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]

    def run(mode):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        ev0.record(streams[0])
        streams[1].wait_event(ev0)
        for _ in range(args.iters):
            for u, (ana, syn, x, chan, out) in enumerate(units):
                s = streams[0] if mode == "serial" else streams[u]
                with torch.cuda.stream(s):
                    pfb.roundtrip(ana, syn, x, chan=chan, out=out)
        done = torch.cuda.Event()
        done.record(streams[1])
        streams[0].wait_event(done)
        ev1.record(streams[0])
        torch.cuda.synchronize()
        return ev0.elapsed_time(ev1) * 1e3 / (2 * args.iters)

    for mode in ("serial", "conc"):
        run(mode)
    res = {"tag": args.tag, "env": {k: v for k, v in os.environ.items() if k.startswith("PFB_") and k != "PFB_HIP_LIB"}}
    for mode in ("serial", "conc", "serial", "conc"):
        ts = [run(mode) for _ in range(args.reps)]
        res.setdefault(mode, []).append(round(float(np.median(ts)), 1))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
