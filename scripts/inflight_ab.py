"""A/B of the C2 round trip with D steps in flight (development tool; any library build).

The bench.py timed loop in miniature: D (analysis, synthesis) plan pairs, each step one
HIP-graph replay of pfb_roundtrip_execute on its pair's stream (step i -> pair i mod D),
K steps between device synchronizes.  Unlike bench.py it runs whatever library
PFB_HIP_LIB names, so the experiments build's launch-geometry knobs (PFB_ANA_WG_PER_CU,
PFB_WAVE_PER_CU, ...) can be compared in the in-flight regime.  Prints one JSON line:
microseconds per step (median of --reps timings).

    PFB_HIP_LIB=ska-pst-dsp-model_amd/lib/libpfb_hip_exp.so PFB_ANA_WG_PER_CU=1 \\
        python scripts/inflight_ab.py --tag ana1 --inflight 3
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ska-pst-dsp-model_amd"), REPO]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="")
    ap.add_argument("--inflight", type=int, default=3)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--n-pol", type=int, default=1)
    ap.add_argument("--pipeline", type=int, default=0,
                    help="1: the K steps as bench.py's captured two-stream pipeline (capture_pipeline); "
                         "2: the K steps captured in order on ONE stream as one graph")
    args = ap.parse_args()
    import torch
    import ska_pst_dsp_model_amd as pfb
    from ska_pst_dsp_model_amd import _lib
    dev = torch.device("cuda", 0)
    taps = pfb.design_PFB_FIR_filter(256, "8/7", 12)
    g = torch.Generator(device=dev).manual_seed(100)
    n = 1 << 24

    def noise():
        return (torch.complex(torch.randn((args.n_pol, n), device=dev, generator=g),
                              torch.randn((args.n_pol, n), device=dev, generator=g)) / np.sqrt(2)).to(torch.complex64)
    win = pfb.PFBWindow().lookup["tukey"](256, 48)
    D = max(1, args.inflight)
    graphs, streams = [], [torch.cuda.Stream(dev) for _ in range(D)]
    keep = []  # the plans and buffers each captured graph writes stay alive while it replays
    for _ in range(D):
        x = noise()  # distinct inputs per pair, as bench.py's units (none stays cache-resident)
        ana = pfb.AnalysisPlan(taps, 256, "8/7", "polyphase_analysis", args.n_pol, 0)
        syn = pfb.SynthesisPlan(256, "8/7", 256, 48, True, 1, True, taps, win, None, args.n_pol, 0)
        K = ana.output_length(n)
        chan = torch.empty((args.n_pol, K, 256), dtype=torch.complex64, device=dev)
        out = torch.empty((args.n_pol, syn.output_length(K)), dtype=torch.complex64, device=dev)

        keep.append((ana, syn, chan, out, x))

        def step(ana=ana, syn=syn, chan=chan, out=out, x=x):
            pfb.roundtrip(ana, syn, x, chan=chan, out=out)
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            step()
        torch.cuda.synchronize()
        graphs.append(gr)

    if args.pipeline:
        # bench.py's timed region: one replay of the K steps as a captured two-stream
        # pipeline (step i's analysis beside step i-1's synthesis)
        sys.path.insert(0, REPO)
        from bench import capture_pipeline
        pairs = [(k[0], k[1], k[2], k[3]) for k in keep]
        inputs = [k[4] for k in keep]
        if args.pipeline == 1:
            batch = capture_pipeline(torch, dev, pfb, pairs, inputs, n, args.steps)
        else:
            g1 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1):
                for i in range(args.steps):
                    a_, s_, c_, o_ = pairs[i % D]
                    pfb.roundtrip(a_, s_, inputs[i % D], chan=c_, out=o_)
            torch.cuda.synchronize()
            batch = g1.replay
        batch()
        torch.cuda.synchronize()

        def run_pipe():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            batch()
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) * 1e6 / args.steps
        ts = [run_pipe() for _ in range(args.reps)]
        print(json.dumps({"tag": args.tag, "lib": os.path.basename(_lib.LIB_PATH), "inflight": D,
                          "pipeline": args.pipeline, "n_pol": args.n_pol,
                          "env": {k: v for k, v in os.environ.items() if k.startswith("PFB_") and k != "PFB_HIP_LIB"},
                          "us_per_step": round(float(np.median(ts)), 1),
                          "us_all": [round(t, 1) for t in ts]}), flush=True)
        return

    def run(k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(k):
            with torch.cuda.stream(streams[i % D]):
                graphs[i % D].replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6 / k

    run(2 * D)
    ts = [run(args.steps) for _ in range(args.reps)]
    print(json.dumps({"tag": args.tag, "lib": os.path.basename(_lib.LIB_PATH), "inflight": D,
                      "n_pol": args.n_pol,
                      "env": {k: v for k, v in os.environ.items() if k.startswith("PFB_") and k != "PFB_HIP_LIB"},
                      "us_per_step": round(float(np.median(ts)), 1),
                      "us_all": [round(t, 1) for t in ts]}), flush=True)


if __name__ == "__main__":
    main()
