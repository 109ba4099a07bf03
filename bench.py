"""Benchmark: PFB analysis -> synthesis round trip, complex Msamples/s (BASELINE.json).

One step = one pass of the hot path over one unit of synthetic input resident in HBM:
``polyphase_analysis`` (SKA-Low, 256 channels, OS 8/7, 3073 firls taps) of 2^24
complex samples followed by ``polyphase_synthesis`` (Nf 256, Ov 48, tukey, deripple
on, spans Nyquist) of the channelised output — BASELINE config C2 (configs[1]).

Multi-GPU (``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N``):
one process per GPU, each processes its own independent unit (time block /
polarisation; BASELINE C4 sharding) — no collective on the data path.  Timing is
bracketed by a barrier + device synchronize and the max over ranks is reported.

Rank 0 prints one JSON line with the throughput, the roofline of the dominant kernel
(HIP events on the library's launch stream, algorithmic bytes per launch) and the CPU
baseline (the NumPy oracle on a bounded sample, single core).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(REPO, "ska-pst-dsp-model_amd"), REPO]

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

N_CHAN, OS_STR, TAPS_PER_CHAN = 256, "8/7", 12
NF, OV = 256, 48
N_DAT = 1 << 24


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n-dat", type=int, default=N_DAT)
    ap.add_argument("--n-pol", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--chunk-blocks", type=int, default=0)
    ap.add_argument("--graph", type=int, default=1,
                    help="capture one step (3 kernel launches) in a HIP graph and replay it")
    ap.add_argument("--roundtrip", type=int, default=1,
                    help="1: one pfb_roundtrip_execute call per step (the analysis kernel also "
                         "runs the synthesis channel IFFT on the rows it produces; the "
                         "channelised product is still written in full); 0: separate "
                         "analysis and synthesis calls")
    ap.add_argument("--kernel-events", type=int, default=1,
                    help="record HIP events around every kernel in the timed region")
    ap.add_argument("--e2e", type=int, default=0,
                    help="also time the host-buffer path: pinned DADA bytes (NBIT 8 TFP) -> "
                         "H2D -> unpack -> round trip -> pack (NBIT 32) -> D2H (reported as "
                         "e2e_pcie; never the headline value)")
    return ap.parse_args()


def cpu_baseline(taps, budget_s: float):
    """Time the oracle (NumPy restatement, complex64 like Matlab single) on a bounded
    sample of the same workload: 2^20-sample units, repeated for ~budget_s seconds."""
    from oracle import pfb_oracle as orc
    n = 1 << 20
    rng = np.random.default_rng(0)
    x = ((rng.standard_normal((1, 1, n)) + 1j * rng.standard_normal((1, 1, n))) /
         np.sqrt(2)).astype(np.complex64)
    win = orc.pfb_window("tukey", NF, OV)
    dr = {"apply_deripple": 1, "filter_coeff": taps}
    reps, t0 = 0, time.perf_counter()
    while True:
        chan = orc.polyphase_analysis(x, taps, N_CHAN, OS_STR, dtype=np.complex64)
        orc.polyphase_synthesis(chan, 1, NF, OS_STR, dr, 1, OV, win, dtype=np.complex64)
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s or reps >= 4096:
            break
    return {
        "value": reps * n / el / 1e6,
        "unit": "complex Msamples/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{reps} x 2^20-sample units of the C2 workload (NumPy oracle, complex64, "
                  f"numpy.fft single-threaded), {el:.1f} s",
    }


def copy_rate(torch, dev, lib, n_bytes: int = 1 << 31, reps: int = 20):
    """Achievable HBM bandwidth on this device ("also measure achievable
    bandwidth with a device copy kernel and report both"): the library's float4 copy
    kernel (pfb_device_copy) over n_bytes, counted as n_bytes read + n_bytes written,
    median over reps, HIP events on the stream the kernel runs on."""
    src = torch.empty(n_bytes // 4, dtype=torch.float32, device=dev).fill_(1.0)
    dst = torch.empty_like(src)
    stream = torch.cuda.current_stream(dev)

    def copy():
        if lib.pfb_device_copy(dst.data_ptr(), src.data_ptr(), n_bytes, stream.cuda_stream):
            raise RuntimeError(lib.pfb_last_error().decode())

    for _ in range(3):
        copy()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        copy()
        e1.record(stream)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = float(np.median(ts))
    ok = bool(torch.equal(dst[:1 << 20], src[:1 << 20]))
    del src, dst
    return round(2.0 * n_bytes / (ms * 1e-3) / 1e9, 1) if ok else None


def pmc_traffic():
    """HBM bytes per launch per kernel class from the committed PMC summary
    (scripts/pmc_summary.py --json, FETCH_SIZE/WRITE_SIZE passes), if any."""
    p = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            return json.load(f)
    except Exception:
        return None


def e2e_pcie(torch, dev, pfb, ana, syn, n_pol, n_dat, chan_buf, out_buf, steps, world, dist):
    """Host-buffer rate of the DADA path: int8 TFP bytes in pinned host
    memory -> H2D -> pfb_dada_unpack -> round trip -> pfb_dada_pack (float32) -> D2H into
    pinned memory, one unit per step, serial on one stream."""
    from ska_pst_dsp_model_amd import layout
    rng = np.random.default_rng(5)
    raw_h = torch.from_numpy(rng.integers(-40, 40, size=n_dat * n_pol * 2, dtype=np.int8)
                             .view(np.uint8)).pin_memory()
    n_out = out_buf.shape[1]
    res_h = torch.empty((n_out * n_pol * 2,), dtype=torch.float32).pin_memory()
    raw_d = torch.empty_like(raw_h, device=dev)

    def step():
        raw_d.copy_(raw_h, non_blocking=True)
        x = layout.dada_unpack(raw_d, 8, 2, 1, n_pol)[:, :, 0]       # (n_pol, n_dat)
        pfb.roundtrip(ana, syn, x, chan=chan_buf, out=out_buf)
        packed = layout.dada_pack(out_buf[:, :, None], 32)
        res_h.copy_(packed, non_blocking=True)

    step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    return {"value": round(n_pol * n_dat * steps / el / 1e6, 2), "unit": "complex Msamples/s",
            "per_gpu": True, "input": "DADA NBIT 8 TFP, pinned host memory",
            "output": "DADA NBIT 32 TFP, pinned host memory", "ms_per_step": round(el / steps * 1e3, 3)}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    import ska_pst_dsp_model_amd as pfb
    from ska_pst_dsp_model_amd import _lib

    taps = pfb.design_PFB_FIR_filter(N_CHAN, OS_STR, TAPS_PER_CHAN)
    n_pol, n_dat = args.n_pol, args.n_dat
    # independent unit per rank (seed = 100 + rank, BASELINE C4 seeds)
    g = torch.Generator(device=dev).manual_seed(100 + rank)
    x = torch.complex(torch.randn((n_pol, n_dat), device=dev, generator=g),
                      torch.randn((n_pol, n_dat), device=dev, generator=g)) / np.sqrt(2.0)
    x = x.to(torch.complex64).contiguous()

    ana = pfb.AnalysisPlan(taps, N_CHAN, OS_STR, "polyphase_analysis", n_pol, local)
    win = pfb.PFBWindow().lookup["tukey"](NF, OV)
    syn = pfb.SynthesisPlan(N_CHAN, OS_STR, NF, OV, True, 1, True, taps, win, None, n_pol, local)
    if args.chunk_blocks:
        syn.set_chunk_blocks(args.chunk_blocks)
    K = ana.output_length(n_dat)
    n_out = syn.output_length(K)

    chan_buf = torch.empty((n_pol, K, N_CHAN), dtype=torch.complex64, device=dev)
    out_buf = torch.empty((n_pol, n_out), dtype=torch.complex64, device=dev)

    def step_serial():
        chan = ana.execute(x)            # (n_pol, K, N) time-major channelised data
        return syn.execute(chan, layout="ptc")

    def step_pipelined():
        return pfb.roundtrip(ana, syn, x, chan=chan_buf, out=out_buf)

    step = step_pipelined if args.roundtrip else step_serial

    lib = _lib.load()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    run = step
    if args.graph:
        # the plans own all their device buffers after the warm-up, so the step is
        # capturable: one graph launch replays analysis + channel IFFT + block kernel
        graph = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream(device=dev)
        cs.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(cs):
            step()
        torch.cuda.current_stream(dev).wait_stream(cs)
        with torch.cuda.graph(graph):
            step()
        torch.cuda.synchronize(dev)
        run = graph.replay

    def timed(steps, fn):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    # timed region: K steps, no instrumentation (value, ms_per_step)
    el = timed(args.steps, run)
    # profiled region: the same K steps with HIP events recorded around every kernel
    # launch on the library's launch stream (per-kernel durations for the roofline;
    # the events add inter-kernel gaps, so this region is not used for `value`).  The
    # kernels of a step run one after another on one stream, so a kernel's
    # event-bracketed duration is its own.
    lib.pfb_profile_reset()
    lib.pfb_profile_enable(args.kernel_events)
    el_prof = timed(args.steps, step)
    lib.pfb_profile_enable(0)

    # per-kernel-class event timings (on the library's launch stream)
    import ctypes
    names = ["analysis", "synth_chan_ifft", "synth_block", "analysis+chan_ifft"]
    kern = {}
    for w in range(4):
        ms, nl, by = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
        lib.pfb_profile_read(w, ctypes.byref(ms), ctypes.byref(nl), ctypes.byref(by))
        if nl.value:
            kern[names[w]] = {"avg_ms": ms.value / nl.value, "launches": nl.value,
                              "alg_bytes_per_launch": by.value / nl.value,
                              "ms_per_step": ms.value / args.steps}

    copy_gbs = copy_rate(torch, dev, lib) if rank == 0 else None

    e2e = None
    if args.e2e:
        e2e = e2e_pcie(torch, dev, pfb, ana, syn, n_pol, n_dat, chan_buf, out_buf, args.steps,
                       world, dist)

    if rank == 0:
        samples = world * n_pol * n_dat * args.steps
        value = samples / el / 1e6
        if kern:
            dom = max(kern, key=lambda k: kern[k]["avg_ms"] * kern[k]["launches"])
            kd = kern[dom]
            achieved = kd["alg_bytes_per_launch"] / (kd["avg_ms"] * 1e-3) / 1e9
        else:
            dom, achieved = None, 0.0
        traffic = pmc_traffic()
        roof = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": ((traffic or {}).get(dom) or {}).get("bytes")}
        if copy_gbs:
            # the same achieved rate against the measured device-copy rate (not the peak)
            roof["copy_achievable"] = copy_gbs
            roof["frac_of_copy"] = round(achieved / copy_gbs, 4)
        # round trip as a whole, at B_alg = 16 (1 + nu/de) bytes per input sample
        b_alg = 16.0 * (1.0 + 8.0 / 7.0)
        rt_gbs = value * 1e6 * b_alg / 1e9 / world
        out = {
            "metric": "complex Msamples/s PFB analysis->synthesis",
            "value": round(value, 2),
            "unit": "complex Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic CN(0,1) complex64 noise, HBM-resident, seed 100+rank",
            "config": {"workload": "C2 SKA-Low single-stage: 256 ch, OS 8/7, 3073 firls taps, "
                                   "2^24 samples/unit, Nf 256, Ov 48, tukey, deripple",
                       "n_chan": N_CHAN, "os_factor": OS_STR, "n_taps": len(taps),
                       "n_dat_per_unit": n_dat, "n_pol": n_pol, "units": world * n_pol,
                       "channelised_rows": K, "output_samples_per_unit": n_out,
                       "parallelism": f"{world} independent units, one per GPU (no collective)",
                       "hip_graph": bool(args.graph),
                       "roundtrip_call": bool(args.roundtrip)},
            "roofline": roof,
            "round_trip_hbm_frac": round(rt_gbs / HBM_PEAK_GBS, 4),
            "ms_per_step_with_kernel_events": round(el_prof / args.steps * 1e3, 4),
            "kernels": kern,
        }
        if e2e is not None:
            out["e2e_pcie"] = e2e
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(taps, args.cpu_seconds)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
