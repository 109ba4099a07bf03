"""A/B timing of the C2 round trip's kernels (development tool, experiments build).

Runs the bench.py C2 step (pfb_roundtrip_execute, 2^24 samples) with HIP events on every
kernel launch and prints one JSON line: per kernel class the average duration and the
kernel name.  The library is whatever PFB_HIP_LIB names (default: the release build); the
experiments build (make EXPERIMENTS=1) reads its PFB_* knobs from the environment, so
variants are separate processes:

    PFB_HIP_LIB=ska-pst-dsp-model_amd/lib/libpfb_hip_exp.so PFB_SYNTH_WAVE=0 \\
        python scripts/ab_kernels.py --tag old
"""
import argparse
import ctypes
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
    ap.add_argument("--n-pol", type=int, default=1)
    ap.add_argument("--os", default="8/7")
    args = ap.parse_args()
    import torch
    import ska_pst_dsp_model_amd as pfb
    from ska_pst_dsp_model_amd import _lib
    dev = torch.device("cuda", 0)
    taps = pfb.design_PFB_FIR_filter(256, args.os, 12)
    g = torch.Generator(device=dev).manual_seed(100)
    n = 1 << 24
    x = (torch.complex(torch.randn((args.n_pol, n), device=dev, generator=g),
                       torch.randn((args.n_pol, n), device=dev, generator=g)) / np.sqrt(2)).to(torch.complex64)
    ana = pfb.AnalysisPlan(taps, 256, args.os, "polyphase_analysis", args.n_pol, 0)
    win = pfb.PFBWindow().lookup["tukey"](256, 48)
    syn = pfb.SynthesisPlan(256, args.os, 256, 48, True, 1, True, taps, win, None, args.n_pol, 0)
    K = ana.output_length(n)
    chan = torch.empty((args.n_pol, K, 256), dtype=torch.complex64, device=dev)
    out = torch.empty((args.n_pol, syn.output_length(K)), dtype=torch.complex64, device=dev)
    lib = _lib.load()
    for _ in range(3):
        pfb.roundtrip(ana, syn, x, chan=chan, out=out)
    torch.cuda.synchronize()
    lib.pfb_profile_reset()
    lib.pfb_profile_enable(1)
    for _ in range(args.steps):
        pfb.roundtrip(ana, syn, x, chan=chan, out=out)
    torch.cuda.synchronize()
    lib.pfb_profile_enable(0)
    res = {"tag": args.tag, "lib": os.path.basename(_lib.LIB_PATH),
           "env": {k: v for k, v in os.environ.items() if k.startswith("PFB_") and k != "PFB_HIP_LIB"}}
    for w, name in enumerate(["analysis", "synth_chan_ifft", "synth_block", "analysis+chan_ifft"]):
        ms, nl, by = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
        lib.pfb_profile_read(w, ctypes.byref(ms), ctypes.byref(nl), ctypes.byref(by))
        if nl.value:
            buf = ctypes.create_string_buffer(512)
            lib.pfb_profile_kernel_name(w, buf, len(buf))
            res[name] = {"us": round(ms.value / nl.value * 1e3, 2),
                         "kernel": buf.value.decode().split("(")[0].replace("void pfb::", "")}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
