"""Secondary measurements (not the bench.py headline): every other kernel of the path on
one MI355X, as algorithmic HBM bytes / time against the 8 TB/s peak.

  * C3 SKA-Mid padded round trip (4096 ch, 8/7, 100 353 taps, 2^26 samples)
  * C2' reference 'low' parity variant (256 ch, 4/3)
  * LowCBF PST filterbank (polyphase_analysis_lowcbf, 2^24 samples x 2 pol)
  * DADA unpack (NBIT 8 / 32) and pack, corner turn, channel gather, quantisation
  * two-stage analysis cascade (256 x 256 ch; stage 2 batched over 256 series)

Prints one JSON object per line.  Usage: python scripts/bench_aux.py [--reps N]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ska-pst-dsp-model_amd"), REPO]
PEAK = 8000.0


def timeit(torch, fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def emit(name, ms, alg_bytes, **kw):
    gbs = alg_bytes / (ms * 1e-3) / 1e9
    print(json.dumps({"kernel": name, "ms": round(ms, 4), "alg_bytes": int(alg_bytes),
                      "GB/s": round(gbs, 1), "frac": round(gbs / PEAK, 4), **kw}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--skip-mid", action="store_true")
    ap.add_argument("--only-mid", action="store_true")
    ap.add_argument("--only-twostage", action="store_true")
    ap.add_argument("--inflight", type=int, default=1, help="C3 units in flight (plan pairs/streams)")
    ap.add_argument("--graph", type=int, default=1, help="with --pipeline: capture the steps as one graph")
    ap.add_argument("--pipeline", type=int, default=0,
                    help="with --inflight > 1: the split round trip pipelined over two streams")
    ap.add_argument("--cpu", action="store_true",
                    help="also time the NumPy oracle (1 core) on bounded samples of each config")
    args = ap.parse_args()
    import torch
    import ska_pst_dsp_model_amd as pfb
    from ska_pst_dsp_model_amd import layout
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)

    def noise(*shape):
        return torch.complex(torch.randn(shape, device=dev, generator=g),
                             torch.randn(shape, device=dev, generator=g)).to(torch.complex64)

    if args.cpu:
        cpu_baselines(pfb)
    if args.only_mid:
        return mid(torch, pfb, noise, dev, reps=args.reps, inflight=args.inflight, pipeline=bool(args.pipeline),
                   graph=bool(args.graph))
    if args.only_twostage:
        return twostage(torch, pfb, noise, args.reps)
    # ---- C2' (4/3) round trip
    taps43 = pfb.design_PFB_FIR_filter(256, "4/3", 12)
    n = 1 << 24
    x = noise(1, n)
    ana = pfb.AnalysisPlan(taps43, 256, "4/3", "polyphase_analysis", 1)
    win = pfb.PFBWindow().lookup["tukey"](256, 48)
    syn = pfb.SynthesisPlan(256, "4/3", 256, 48, True, 1, True, taps43, win, None, 1)
    K = ana.output_length(n)
    chan = torch.empty((1, K, 256), dtype=torch.complex64, device=dev)
    out = torch.empty((1, syn.output_length(K)), dtype=torch.complex64, device=dev)
    ms = timeit(torch, lambda: pfb.roundtrip(ana, syn, x, chan=chan, out=out), args.reps)
    emit("roundtrip C2' 256ch 4/3", ms, 16 * (1 + 4 / 3) * n,
         msamples_per_s=round(n / ms / 1e3, 1))

    # ---- LowCBF PST filterbank
    taps_pst = pfb.read_fir_filter_coeff(os.path.join(pfb.config.config_dir, "PST_filtertaps.txt"))
    x2 = noise(2, n)
    low = pfb.AnalysisPlan(taps_pst, 256, "4/3", "polyphase_analysis_lowcbf", 2)
    low.execute(x2)  # consume the one-time padding
    Kl = low.output_length(n)
    ms = timeit(torch, lambda: low.execute(x2), args.reps)
    emit("lowcbf_kernel (PSTFilterbank)", ms, 2 * (8 * n + 8 * 216 * Kl),
         msamples_per_s=round(2 * n / ms / 1e3, 1))

    # ---- layout kernels
    raw8 = torch.randint(-128, 127, (2 * 2 * n,), dtype=torch.int8, device=dev)
    ms = timeit(torch, lambda: layout.dada_unpack(raw8, 8, 2, 1, 2), args.reps)
    emit("dada_unpack NBIT8 2pol", ms, raw8.numel() + 2 * n * 8)
    raw32 = torch.randn((2 * 2 * n,), device=dev)
    ms = timeit(torch, lambda: layout.dada_unpack(raw32, 32, 2, 1, 2), args.reps)
    emit("dada_unpack NBIT32 2pol", ms, raw32.numel() * 4 + 2 * n * 8)
    y = noise(2, n, 1)
    ms = timeit(torch, lambda: layout.dada_pack(y, 32), args.reps)
    emit("dada_pack NBIT32 2pol", ms, 2 * 2 * n * 8)
    rows = noise(1 << 16, 256)
    ms = timeit(torch, lambda: layout.corner_turn(rows), args.reps)
    emit("corner_turn 65536x256", ms, 2 * rows.numel() * 8)
    ms = timeit(torch, lambda: layout.gather_channels(rows, 16, 16, 256, 1 << 16, 16), args.reps)
    emit("gather_channels 16x16", ms, 2 * rows.numel() * 8)
    ms = timeit(torch, lambda: layout.quantize(y, 33.8), args.reps)
    emit("quantize (moments + round)", ms, 3 * y.numel() * 8)

    # ---- two-stage analysis: 256 ch, then 256 ch over each (batched)
    twostage(torch, pfb, noise, 3)

    # ---- C3 SKA-Mid padded round trip
    if not args.skip_mid:
        del x, x2, raw8, raw32, y, rows, chan, out
        torch.cuda.empty_cache()
        mid(torch, pfb, noise, dev)


def twostage(torch, pfb, noise, reps):
    taps87 = pfb.design_PFB_FIR_filter(256, "8/7", 12)
    cfg = dict(analysis_function="polyphase_analysis", filt_coeff=taps87, channels=256,
               os_factor="8/7")
    ts = pfb.TwoStageFilterBank(cfg)
    xs = noise(1, 1, 1 << 24)
    ts.execute(xs)
    ts2 = pfb.TwoStageFilterBank(cfg)
    ms = timeit(torch, lambda: ts2.execute(xs), reps)
    emit("TwoStageFilterBank 256x256 (stream call)", ms, 16 * (1 + 8 / 7) * (1 << 24),
         msamples_per_s=round((1 << 24) / ms / 1e3, 1),
         note="bytes: the two analyses' input+output; strided stores, no corner turn / gather")
    ts3 = pfb.TwoStageFilterBank(cfg)
    ts3.strided = False
    ts3.execute(xs)
    ms = timeit(torch, lambda: ts3.execute(xs), reps)
    emit("TwoStageFilterBank 256x256 (corner turn + gather path)", ms, 16 * (1 + 8 / 7) * (1 << 24),
         msamples_per_s=round((1 << 24) / ms / 1e3, 1),
         note="bytes: the two analyses' input+output, excluding the corner turn and gather")
    del xs, ts, ts2, ts3
    # BASELINE configs[2]'s cascade: both stages polyphase_analysis_padded (test.config.json
    # `mid`, TwoStageFilterBank.m:27,51-52) — the SKA-Mid stage 1 (4096 ch, 8/7, 100 353 taps)
    # into a 16-ch padded stage 2 over every coarse channel, critical, one 2^26-sample unit
    taps1 = pfb.design_PFB_FIR_filter_two_stage(4096, "8/7", 28)
    taps2 = pfb.design_PFB_FIR_filter(16, "8/7", 10)

    def pcfg(t, n):
        return dict(analysis_function="polyphase_analysis_padded", filt_coeff=t, channels=n, os_factor="8/7")
    nm = 1 << 26
    xm = noise(1, 1, nm)
    tm = pfb.TwoStageFilterBank(pcfg(taps1, 4096)).set_stage2_config(pcfg(taps2, 16))
    tm.critical = 1
    tm.execute(xm)
    ms = timeit(torch, lambda: tm.execute(xm), reps)
    emit("TwoStageFilterBank SKA-Mid 4096x16 padded (stream call)", ms, 16 * (1 + 8 / 7) * nm,
         msamples_per_s=round(nm / ms / 1e3, 1),
         note="both stages polyphase_analysis_padded; bytes: the two analyses' input+output")
    del xm, tm


def cpu_baselines(pfb):
    """The reference's CPU path stand-in (the NumPy oracle, complex64 where Matlab uses
    single, numpy.fft single-threaded) on bounded samples of the other configurations."""
    import time
    from oracle import pfb_oracle as orc
    rng = np.random.default_rng(0)

    def noise(n, n_pol=1):
        return ((rng.standard_normal((n_pol, 1, n)) + 1j * rng.standard_normal((n_pol, 1, n))) /
                np.sqrt(2)).astype(np.complex64)

    def timed(fn, samples, what, sample):
        t0 = time.perf_counter()
        fn()
        el = time.perf_counter() - t0
        print(json.dumps({"cpu": what, "msamples_per_s": round(samples / el / 1e6, 3),
                          "cores": 1, "kind": "port", "sample": sample,
                          "seconds": round(el, 2)}), flush=True)

    taps43 = pfb.design_PFB_FIR_filter(256, "4/3", 12)
    x = noise(1 << 20)
    win = orc.pfb_window("tukey", 256, 48)
    dr = {"apply_deripple": 1, "filter_coeff": taps43}
    timed(lambda: orc.polyphase_synthesis(
        orc.polyphase_analysis(x, taps43, 256, "4/3", dtype=np.complex64), 1, 256, "4/3", dr, 1,
        48, win, dtype=np.complex64), 1 << 20, "C2' round trip", "2^20 samples")
    pst = pfb.read_fir_filter_coeff(os.path.join(pfb.config.config_dir, "PST_filtertaps.txt"))
    x2 = noise(1 << 18, 2)
    timed(lambda: orc.polyphase_analysis_lowcbf(x2, pst, do_padding=False), 2 << 18,
          "LowCBF PST filterbank", "2 pol x 2^18 samples")
    tm = pfb.design_PFB_FIR_filter_two_stage(4096, "8/7", 28)
    x3 = noise(1 << 22)
    winm = orc.pfb_window("tukey", 512, 128)
    drm = {"apply_deripple": 1, "filter_coeff": tm}
    timed(lambda: orc.polyphase_synthesis(
        orc.polyphase_analysis_padded(x3, tm, 4096, "8/7", dtype=np.complex64), 1, 512, "8/7",
        drm, 1, 128, winm, dtype=np.complex64), 1 << 22, "C3 SKA-Mid round trip",
        "2^22 samples (2 synthesis blocks)")


def mid(torch, pfb, noise, dev, reps=3, inflight=1, pipeline=False, graph=False):
    tm = pfb.design_PFB_FIR_filter_two_stage(4096, "8/7", 28)
    nm = 1 << 26
    xm = noise(1, nm)
    winm = pfb.PFBWindow().lookup["tukey"](512, 128)
    pairs = []
    for _ in range(max(1, inflight)):
        anam = pfb.AnalysisPlan(tm, 4096, "8/7", "polyphase_analysis_padded", 1)
        synm = pfb.SynthesisPlan(4096, "8/7", 512, 128, True, 1, True, tm, winm, None, 1)
        Km = anam.output_length(nm)
        chm = torch.empty((1, Km, 4096), dtype=torch.complex64, device=dev)
        om = torch.empty((1, synm.output_length(Km)), dtype=torch.complex64, device=dev)
        pairs.append((anam, synm, chm, om))
    # each unit in flight reads its own input (no shared input lines between the units)
    xs = [xm] + [noise(1, nm) for _ in pairs[1:]]
    if len(pairs) == 1:
        anam, synm, chm, om = pairs[0]
        ms = timeit(torch, lambda: pfb.roundtrip(anam, synm, xm, chan=chm, out=om), reps)
    elif pipeline:
        # the split round trip as a two-stream pipeline (bench.py --pipeline): unit i's
        # FIR + row FFT on stream A beside unit i-1's synthesis on stream S
        for (a, s_, c, o), xi in zip(pairs, xs):
            pfb.roundtrip(a, s_, xi, chan=c, out=o)
        torch.cuda.synchronize()
        D = len(pairs)

        def enqueue(k):
            sa = torch.cuda.current_stream()
            ss = torch.cuda.Stream(dev)
            ss.wait_stream(sa)
            ev_a = [torch.cuda.Event() for _ in range(k)]
            ev_s = [torch.cuda.Event() for _ in range(k)]
            for i in range(k):
                a, s_, c, o = pairs[i % D]
                if i >= D:
                    sa.wait_event(ev_s[i - D])
                pfb.roundtrip_analysis(a, s_, xs[i % D], chan=c)
                ev_a[i].record(sa)
                ss.wait_event(ev_a[i])
                with torch.cuda.stream(ss):
                    pfb.roundtrip_synthesis(a, s_, nm, out=o)
                ev_s[i].record(ss)
            sa.wait_stream(ss)
        import time
        n_it = reps * D
        enqueue(D)
        torch.cuda.synchronize()
        if graph:
            # the n_it steps captured as one graph (bench.py's form; eager launches of these
            # persistent kernels on two streams interleave destructively)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                enqueue(n_it)
            g.replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g.replay()
            torch.cuda.synchronize()
        else:
            t0 = time.perf_counter()
            enqueue(n_it)
            torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / n_it
    else:
        # D units in flight: unit i on plan pair i mod D and stream i mod D (no dependence
        # between the pairs), so one unit's FIR / row FFT can run beside another's synthesis
        streams = [torch.cuda.Stream(dev) for _ in pairs]
        ctr = [0]

        def step():
            i = ctr[0] % len(pairs)
            ctr[0] += 1
            a, s_, c, o = pairs[i]
            with torch.cuda.stream(streams[i]):
                pfb.roundtrip(a, s_, xm, chan=c, out=o)

        def sync_all():
            torch.cuda.synchronize()
        for _ in range(len(pairs)):
            step()
        sync_all()
        import time
        n_it = reps * len(pairs)
        t0 = time.perf_counter()
        for _ in range(n_it):
            step()
        sync_all()
        ms = (time.perf_counter() - t0) * 1e3 / n_it
    emit("roundtrip C3 SKA-Mid padded 4096ch", ms, 16 * (1 + 8 / 7) * nm,
         msamples_per_s=round(nm / ms / 1e3, 1), n_taps=len(tm), units_in_flight=len(pairs),
         pipeline=bool(pipeline and len(pairs) > 1), graph=bool(graph and pipeline and len(pairs) > 1))


if __name__ == "__main__":
    main()
