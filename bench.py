"""Benchmark: PFB analysis -> synthesis round trip, complex Msamples/s (BASELINE.json).

One step = one pass of the hot path over one unit of synthetic input resident in HBM:
``polyphase_analysis`` (SKA-Low, 256 channels, OS 8/7, 3073 firls taps) of 2^24
complex samples followed by ``polyphase_synthesis`` (Nf 256, Ov 48, tukey, deripple
on, spans Nyquist) of the channelised output — BASELINE config C2 (configs[1]).

Multi-GPU (BASELINE C4, configs[3]): ``python bench.py --gpus N`` starts N ranks itself
(``torch.distributed.run`` as a child process, before this process makes any GPU call);
under an existing launcher (``torch.distributed.run ... bench.py --gpus N``) WORLD_SIZE
must equal N.  Each rank processes one dual-polarisation DADA time block of the C2
parameters — 2 independent units per GPU, the pols drawn from seeds 100+2r and
100+2r+1 — with no collective on the data path.  Timing is bracketed by
a barrier + device synchronize and the max over ranks is reported;
value = all ranks' samples / that time.  ``--gpus 1`` is the C2 headline (one
single-pol unit, seed 100); ``--workload c4`` runs the C4 unit on one GPU too.

Steps in flight (``--inflight D``, default 3): the units are independent, so a rank keeps D
plan pairs — each with its own stage-1-row scratch, channelised and output buffers and
(``--distinct-inputs``, default) its own synthetic units.  With ``--pipeline 1`` (default)
the K timed steps are one captured two-stream software pipeline: step i's analysis half
(``pfb_roundtrip_analysis_execute``) on stream A, its synthesis half on stream S after an
event, step i's analysis waiting for step i-D's synthesis (the pair's rows are free again)
— so step i+1's analysis runs beside step i's synthesis; ``--pipeline 0`` deals per-step
graphs round-robin over D streams instead.  Every step is still one full analysis +
synthesis of one unit.  The timed region is unchanged: the K steps (one replay of the
captured pipeline) between barrier + synchronize.  The kernel-event region that feeds
``roofline`` runs the steps one at a time (pair 0).

Rank 0 prints one JSON line with the throughput, the roofline of the dominant kernel
(HIP events on the library's launch stream, algorithmic bytes per launch) and, at N=1,
the CPU baseline (the NumPy oracle on a bounded sample, on one core and on all the
host cores the box gives this process).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
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
    ap.add_argument("--workload", choices=("auto", "c2", "c4"), default="auto",
                    help="auto: C2 at --gpus 1, C4 (one dual-pol unit pair per GPU) above")
    ap.add_argument("--cpu-workers", type=int, default=0,
                    help="processes of the all-cores CPU leg (0: the cores this process may use)")
    ap.add_argument("--stub-device", action="store_true",
                    help="test hook: replace the device step by a CPU no-op and use gloo "
                         "(exercises the launcher, unit mapping and aggregation without a GPU)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n-dat", type=int, default=N_DAT)
    ap.add_argument("--n-pol", type=int, default=0, help="override the workload's pols per rank")
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
    ap.add_argument("--inflight", type=int, default=3,
                    help="steps in flight: D plan pairs (each with its own stage-1-row, "
                         "channelised and output buffers) on D streams, step i on pair i mod D, "
                         "so one step's analysis can run beside the previous step's synthesis")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="with --inflight D > 1: the K timed steps as one captured two-stream "
                         "pipeline (pfb_roundtrip_analysis_execute on stream A, "
                         "pfb_roundtrip_synthesis_execute on stream S, events between); 0: "
                         "per-step graphs dealt round-robin over D streams")
    ap.add_argument("--distinct-inputs", type=int, default=1,
                    help="with --inflight D > 1: every plan pair reads its own synthetic units "
                         "(seeds + 7919 p), so overlapping steps share no input data")
    ap.add_argument("--kernel-events", type=int, default=1,
                    help="record HIP events around every kernel in the timed region")
    ap.add_argument("--stage1", choices=("auto", "stored", "recomputed"), default="auto",
                    help="synthesis stage-1 rows of the fused round trip "
                         "(pfb_synthesis_set_stage1_rows): written by the analysis and read back, "
                         "or recomputed from the input by the synthesis (bit-identical output)")
    ap.add_argument("--c3", type=int, default=1,
                    help="N=1 only: also time BASELINE configs[2] (C3 SKA-Mid padded round trip, "
                         "4096 ch, 100 353 taps, 2^26 samples) as the line's `c3` key (not the "
                         "headline value)")
    ap.add_argument("--synthesis-only", type=int, default=1,
                    help="N=1 only: also time the standalone synthesis of an HBM-resident C2 "
                         "channelised product (SynthesisPlan.execute: channel IFFT + synthesis, "
                         "the PST InverseFilterBank case) as the line's `synthesis_only` key")
    ap.add_argument("--e2e", type=int, default=0,
                    help="also time the host-buffer path: pinned DADA bytes (NBIT 8 TFP) -> "
                         "H2D -> unpack -> round trip -> pack (NBIT 32) -> D2H (reported as "
                         "e2e_pcie; never the headline value)")
    return ap.parse_args()


CPU_UNIT = 1 << 20  # samples per CPU-baseline unit (a bounded sample of the C2 workload)


def _cpu_unit_loop(budget_s: float, taps, seed: int = 0, barrier=None):
    """Oracle round trips of 2^20-sample C2 units (NumPy, complex64 like Matlab single,
    numpy.fft) for ~budget_s seconds in this process -> (units, seconds)."""
    from oracle import pfb_oracle as orc
    rng = np.random.default_rng(seed)
    x = ((rng.standard_normal((1, 1, CPU_UNIT)) + 1j * rng.standard_normal((1, 1, CPU_UNIT))) /
         np.sqrt(2)).astype(np.complex64)
    win = orc.pfb_window("tukey", NF, OV)
    dr = {"apply_deripple": 1, "filter_coeff": taps}
    if barrier is not None:
        barrier.wait()  # all workers start their timed loops together
    reps, t0 = 0, time.perf_counter()
    while True:
        chan = orc.polyphase_analysis(x, taps, N_CHAN, OS_STR, dtype=np.complex64)
        orc.polyphase_synthesis(chan, 1, NF, OS_STR, dr, 1, OV, win, dtype=np.complex64)
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s or reps >= 4096:
            return reps, el


_POOL_BARRIER = None


def _pool_init(barrier):
    global _POOL_BARRIER
    _POOL_BARRIER = barrier


def _pool_worker(a):
    # the oracle is NumPy elementwise maths + pocketfft: single-threaded per process
    budget_s, taps, seed = a
    return _cpu_unit_loop(budget_s, taps, seed, _POOL_BARRIER)


def host_info():
    """CPU model and core counts of the machine this runs on (the GPU box's host)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        usable = os.cpu_count()
    omp = os.environ.get("OMP_NUM_THREADS")
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": usable,
            "omp_num_threads": int(omp) if omp and omp.isdigit() else None}


def cpu_workers_default() -> int:
    """The cores this process may use: its affinity set, capped by OMP_NUM_THREADS
    (the GPU box's CPU share for one GPU is 16; nproc shows the whole machine)."""
    h = host_info()
    n = h["affinity_cpus"] or 1
    if h["omp_num_threads"]:
        n = min(n, h["omp_num_threads"])
    return max(1, n)


def cpu_baseline(budget_s: float, workers: int):
    """The oracle (``kind: port`` — the reference is Matlab, nothing of it runs here) on
    a bounded sample of the C2 workload, timed on this host's cores:
    * one core: one process, numpy.fft (pocketfft, single-threaded);
    * all cores: ``workers`` processes, each running the same single-threaded oracle on
      its own 2^20-sample units (the units are independent, as on the GPU), started
      before this process touches the GPU; throughput = all units / wall time.
    The headline ``value``/``cores`` is the all-cores leg; ``single_core`` beside it."""
    import multiprocessing as mp
    from ska_pst_dsp_model_amd import firio
    taps = firio.design_PFB_FIR_filter(N_CHAN, OS_STR, TAPS_PER_CHAN)
    reps1, el1 = _cpu_unit_loop(budget_s, taps)
    one = {"value": reps1 * CPU_UNIT / el1 / 1e6, "cores": 1,
           "sample": f"{reps1} x 2^20-sample C2 units, {el1:.1f} s"}
    out = {"unit": "complex Msamples/s", "kind": "port", "host": host_info(),
           "single_core": one}
    if workers > 1:
        ctx = mp.get_context("fork")
        with ctx.Pool(workers, initializer=_pool_init, initargs=(ctx.Barrier(workers),)) as pool:
            res = pool.map(_pool_worker, [(budget_s, taps, 1000 + i) for i in range(workers)],
                           chunksize=1)
        wall = max(el for _, el in res)  # timed loops start together (barrier)
        units = sum(r for r, _ in res)
        out.update(value=units * CPU_UNIT / wall / 1e6, cores=workers,
                   sample=f"{units} x 2^20-sample C2 units (NumPy oracle round trip, complex64) "
                          f"over {workers} single-threaded processes, {wall:.1f} s wall")
    else:
        out.update(value=one["value"], cores=1, sample=one["sample"] + " (NumPy oracle, 1 core)")
    return out


C3_N_CHAN, C3_TAPS_PER_CHAN, C3_NF, C3_OV = 4096, 28, 512, 128
C3_N_DAT = 1 << 26
C3_CPU_UNIT = 1 << 22  # bounded CPU sample of C3: 2^22 samples = 2 synthesis blocks


def c3_taps():
    from ska_pst_dsp_model_amd import firio
    return firio.design_PFB_FIR_filter_two_stage(C3_N_CHAN, OS_STR, C3_TAPS_PER_CHAN)


def cpu_baseline_c3(taps):
    """The oracle's C3 round trip (polyphase_analysis_padded -> polyphase_synthesis,
    complex64, numpy.fft, one core) on a bounded 2^22-sample sample of the C3 unit."""
    from oracle import pfb_oracle as orc
    rng = np.random.default_rng(3)
    x = ((rng.standard_normal((1, 1, C3_CPU_UNIT)) + 1j * rng.standard_normal((1, 1, C3_CPU_UNIT))) /
         np.sqrt(2)).astype(np.complex64)
    win = orc.pfb_window("tukey", C3_NF, C3_OV)
    dr = {"apply_deripple": 1, "filter_coeff": taps}
    t0 = time.perf_counter()
    chan = orc.polyphase_analysis_padded(x, taps, C3_N_CHAN, OS_STR, dtype=np.complex64)
    orc.polyphase_synthesis(chan, 1, C3_NF, OS_STR, dr, 1, C3_OV, win, dtype=np.complex64)
    el = time.perf_counter() - t0
    return {"value": round(C3_CPU_UNIT / el / 1e6, 3), "unit": "complex Msamples/s", "cores": 1,
            "kind": "port", "sample": f"one 2^22-sample C3 unit (2 synthesis blocks), NumPy oracle "
                                      f"round trip, complex64, {el:.1f} s"}


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


PMC_TRAFFIC = os.path.join(REPO, "profiles", "pmc_traffic.json")


def kernel_key(name):
    """Kernel name as the PMC summary keys it: the demangled template-id without the
    return type, namespace and parameter list ("synth_block_kernel<256, 224, ...>")."""
    if not name:
        return None
    return name.split("(")[0].replace("void ", "").replace("pfb::", "").strip()


def pmc_traffic(path=PMC_TRAFFIC):
    """HBM bytes per launch, per workload and kernel, from the committed PMC summary
    (scripts/pmc_summary.py --json, FETCH_SIZE/WRITE_SIZE passes over bench.py)."""
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        return json.load(f)


# why a kernel's measured HBM bytes exceed 1.6x its algorithmic bytes (bench `traffic_note`)
TRAFFIC_NOTES = {
    "analysis_stream_kernel<256, 13, 8, 7, 2, false, 0>":
        "the fused round trip's analysis also writes the synthesis stage-1 rows (153 MB per unit) "
        "that the algorithmic count (input in + channelised product out) leaves out",
}


def traffic_for(workload, kernel, traffic):
    """(bytes, None) of the PMC record whose kernel IS the timed kernel, else (None, why)."""
    key = kernel_key(kernel)
    if key is None:
        return None, "no kernel name recorded for the dominant kernel class"
    # (stored names are normalised the same way: "pfb::" qualifiers and all)
    recs = {kernel_key(k) or k: v for k, v in (traffic.get(workload) or {}).items()}
    rec = recs.get(key)
    if rec is None:
        return None, f"profiles/pmc_traffic.json has no {workload} record for {key}"
    return rec["bytes"], None


# PFB_* variables that mean nothing to the release library but would change what an
# experiments build times (A/B knobs, timing masks that drop loads/stores): refused
ENV_ALLOWED = {"PFB_PARITY_LOG"}


def pfb_env():
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith("PFB_")}


def check_env():
    bad = sorted(k for k in pfb_env() if k not in ENV_ALLOWED)
    if bad:
        sys.exit(f"bench.py: refusing to run with {', '.join(bad)} set: the benchmark times the "
                 f"release library with no A/B knob or timing mask (unset them)")


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


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n: int) -> int:
    """--gpus N without a launcher: start N ranks with torch.distributed.run as a CHILD
    process (this process has made no GPU call) and return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def resolve_workload(args, world: int) -> str:
    if args.workload != "auto":
        return args.workload
    return "c2" if world == 1 else "c4"


def pair_seeds(seeds, inflight: int, distinct: bool):
    """Seeds of every unit a rank's timed region processes: plan pair p (of the D steps in
    flight) reads units seeds + 7919 p with --distinct-inputs, else pair 0's units."""
    D = max(1, inflight)
    return [sd + (7919 * p if distinct else 0) for p in range(D) for sd in seeds]


def rank_units(workload: str, rank: int):
    """Seeds of the independent units (one per polarisation) rank `rank` processes:
    C2 one single-pol unit (seed 100 + rank); C4 one dual-pol DADA time block = 2 units,
    seeds 100 + 2 rank and 100 + 2 rank + 1 (16 units, seeds 100..115,
    2 per GPU on 8 GPUs)."""
    if workload == "c2":
        return [100 + rank]
    if workload == "c4":
        return [100 + 2 * rank, 100 + 2 * rank + 1]
    raise ValueError(workload)


WORKLOAD_NAMES = {
    "c2": "C2 SKA-Low single-stage: 256 ch, OS 8/7, 3073 firls taps, 2^24 samples/unit, "
          "Nf 256, Ov 48, tukey, deripple; 1 single-pol unit per GPU",
    "c4": "C4 dual-pol SKA-Low 256 ch (C2 parameters): one dual-pol DADA time block of 2^24 "
          "samples per GPU = 2 independent units per GPU, seeds 100+2r, 100+2r+1",
}


def main():
    args = parse()
    check_env()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(env_world or "1")
    if args.gpus != world:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    workload = resolve_workload(args, world)
    seeds = rank_units(workload, rank)
    n_pol = args.n_pol or len(seeds)
    seeds = (seeds * n_pol)[:n_pol] if args.n_pol else seeds
    n_dat = args.n_dat

    # CPU baseline first (rank 0, N = 1), before this process touches the GPU: its
    # worker processes are forked from a process with no device state
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_seconds, args.cpu_workers or cpu_workers_default())
    # C3 (N = 1 only): its taps (plan-time firls design, a few seconds) and its CPU leg
    c3 = None
    if world == 1 and args.c3 and not args.stub_device:
        c3 = {"taps": c3_taps()}
        if not args.no_cpu_baseline:
            c3["cpu_baseline"] = cpu_baseline_c3(c3["taps"])

    import torch
    import torch.distributed as dist

    if args.stub_device:
        if world > 1:
            dist.init_process_group("gloo")
        res = run_stub(args, world, dist)
    else:
        if world > 1:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        res = run_device(args, torch, dist, world, rank, local, n_pol, n_dat, seeds, c3)

    all_seeds = gather_seeds(dist, world, pair_seeds(seeds, args.inflight, args.distinct_inputs),
                             args.stub_device, torch, local)
    if rank == 0:
        out = report(args, res, world, workload, n_pol, n_dat, all_seeds)
        out["cpu_baseline"] = cpu
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def gather_seeds(dist, world, seeds, stub, torch, local):
    if world == 1:
        return [seeds]
    dev = torch.device("cpu") if stub else torch.device("cuda", local)
    t = torch.tensor(seeds, dtype=torch.int64, device=dev)
    buf = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(buf, t)
    return [b.cpu().tolist() for b in buf]


def timed_region(steps, fn, world, dist, sync):
    """K steps bracketed by barrier + device synchronize on both sides; max over ranks."""
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    sync()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        el = max_over_ranks(el, dist)
    return el


def max_over_ranks(el, dist):
    import torch
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" \
        else torch.device("cpu")
    t = torch.tensor([el], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def run_stub(args, world, dist):
    """Device step replaced by a fixed CPU wait (test hook for the launcher)."""
    def step():
        time.sleep(0.002)
    for _ in range(args.warmup):
        step()
    el = timed_region(args.steps, step, world, dist, lambda: None)
    return {"el": el, "el_prof": el, "el_serial": el, "kern": {}, "copy_gbs": None, "e2e": None,
            "taps": 3073, "K": 0, "n_out": 0}


PROFILE_CLASSES = ["analysis", "synth_chan_ifft", "synth_block", "analysis+chan_ifft", "fir", "row_fft"]


def read_profile(lib, steps):
    """Per-kernel-class HIP-event timings recorded since pfb_profile_reset (on the
    library's launch stream): {class: {kernel, avg_ms, launches, alg_bytes_per_launch,
    ms_per_step}}."""
    import ctypes
    kern = {}
    for w, name in enumerate(PROFILE_CLASSES):
        ms, nl, by = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
        lib.pfb_profile_read(w, ctypes.byref(ms), ctypes.byref(nl), ctypes.byref(by))
        if nl.value:
            buf = ctypes.create_string_buffer(512)
            lib.pfb_profile_kernel_name(w, buf, len(buf))
            kern[name] = {"kernel": buf.value.decode() or None,
                          "avg_ms": ms.value / nl.value, "launches": nl.value,
                          "alg_bytes_per_launch": by.value / nl.value,
                          "ms_per_step": ms.value / steps}
    return kern


def capture_pipeline(torch, dev, pfb, pairs, inputs, n_dat, steps):
    """The K steps as ONE captured two-stream software pipeline over D plan pairs: step i's
    analysis half (pfb_roundtrip_analysis_execute) on stream A after step i-D's synthesis
    released pair i mod D's stage-1 rows, its synthesis half
    (pfb_roundtrip_synthesis_execute) on stream S after it — so step i+1's analysis runs
    beside step i's synthesis.  Every step is one full round trip of one unit.  Returns the
    graph's replay."""
    D = len(pairs)

    def enqueue(k):
        sa = torch.cuda.current_stream(dev)
        ss = torch.cuda.Stream(device=dev)
        ss.wait_stream(sa)
        ev_a = [torch.cuda.Event() for _ in range(k)]
        ev_s = [torch.cuda.Event() for _ in range(k)]
        for i in range(k):
            p = i % D
            a_, s_, c_, o_ = pairs[p]
            if i >= D:
                sa.wait_event(ev_s[i - D])
            pfb.roundtrip_analysis(a_, s_, inputs[p], chan=c_)
            ev_a[i].record(sa)
            ss.wait_event(ev_a[i])
            with torch.cuda.stream(ss):
                pfb.roundtrip_synthesis(a_, s_, n_dat, out=o_)
            ev_s[i].record(ss)
        sa.wait_stream(ss)
    pipe = torch.cuda.CUDAGraph()
    with torch.cuda.graph(pipe):
        enqueue(steps)
    torch.cuda.synchronize(dev)
    return pipe.replay


def capture_step(torch, dev, fn):
    """One step captured as a HIP graph (after an eager run on a side stream)."""
    graph = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream(device=dev)
    cs.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(cs):
        fn()
    torch.cuda.current_stream(dev).wait_stream(cs)
    with torch.cuda.graph(graph):
        fn()
    torch.cuda.synchronize(dev)
    return graph.replay


def capture_chain(torch, dev, fns):
    """The calls ``fns`` one after another on one stream, captured as ONE graph (after an
    eager run of each on a side stream): a replay runs them back to back with no graph-launch
    gap between them (a per-step replay leaves ~15 us between steps: the C3 kernel trace,
    profiles/r06_v13_c3_step_trace.json).  Returns the graph's replay."""
    graph = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream(device=dev)
    cs.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(cs):
        for fn in fns:
            fn()
    torch.cuda.current_stream(dev).wait_stream(cs)
    with torch.cuda.graph(graph):
        for fn in fns:
            fn()
    torch.cuda.synchronize(dev)
    return graph.replay


def measure_c3(args, torch, dist, world, dev, pfb, lib, c3, n_pol=1):
    """BASELINE configs[2]: SKA-Mid padded round trip — 4096 channels, OS
    8/7, 100 353 two-stage firls taps, 2^26 samples, Nf 512, Ov 128, tukey, deripple —
    through pfb_roundtrip_execute (FIR -> row FFT -> synthesis), input resident in HBM.
    K timed steps between barrier + synchronize, then the same K with HIP events around
    every kernel (per-kernel durations and the roofline).  n_pol = 2: the SKA-Mid `mid`
    sub-config's dual-polarisation unit (config/test.config.json:104-128), one launch per
    kernel for both pols (the `dual_pol` key; the per-replay and pipelined regions skipped)."""
    taps = c3["taps"]
    win = pfb.PFBWindow().lookup["tukey"](C3_NF, C3_OV)
    D = max(1, args.inflight)
    # D plan pairs, each with its own unit (seed 300 + 7919 p), stage-1 rows, channelised and
    # output buffers: consecutive steps are independent units, as in the C2 headline
    pairs, inputs = [], []
    for p in range(D):
        g = torch.Generator(device=dev).manual_seed(300 + 7919 * p)
        inputs.append((torch.complex(torch.randn((n_pol, C3_N_DAT), device=dev, generator=g),
                                     torch.randn((n_pol, C3_N_DAT), device=dev, generator=g)) /
                       np.sqrt(2.0)).to(torch.complex64))
        ana = pfb.AnalysisPlan(taps, C3_N_CHAN, OS_STR, "polyphase_analysis_padded", n_pol, dev.index or 0)
        syn = pfb.SynthesisPlan(C3_N_CHAN, OS_STR, C3_NF, C3_OV, True, 1, True, taps, win, None, n_pol,
                                dev.index or 0)
        K = ana.output_length(C3_N_DAT)
        n_out = syn.output_length(K)
        pairs.append((ana, syn, torch.empty((n_pol, K, C3_N_CHAN), dtype=torch.complex64, device=dev),
                      torch.empty((n_pol, n_out), dtype=torch.complex64, device=dev)))

    def step_of(p):
        ana, syn, chan, out = pairs[p]
        return lambda: pfb.roundtrip(ana, syn, inputs[p], chan=chan, out=out)
    steps = [step_of(p) for p in range(D)]
    for i in range(max(D, args.warmup)):
        steps[i % D]()
    torch.cuda.synchronize(dev)
    sync = lambda: torch.cuda.synchronize(dev)  # noqa: E731
    # timed region (`ms`): the K steps, step i on pair i mod D (its own unit), one after
    # another on one stream, captured as ONE graph: no graph-launch gap between steps.  The
    # captured two-stream pipeline of the C2 headline (`ms_pipelined`, D > 1) measured SLOWER
    # for C3 (0.862 vs 0.810 ms, r06_v4): its FIR beside the Nf 512 synthesis contends for the
    # CUs that kernel is bound by.  `ms_per_replay`: one graph replay per step (round 6 before
    # the chain: ~15 us of launch gap per step in the kernel trace, r06_v13_c3_step_trace.json).
    chain = capture_chain(torch, dev, [steps[i % D] for i in range(args.steps)])
    el = timed_region(1, chain, world, dist, sync)
    del chain
    el_replay = el_pipe = None
    if n_pol == 1:
        ones = [capture_step(torch, dev, st) for st in steps]
        ctr = [0]

        def one():
            ones[ctr[0] % D]()
            ctr[0] += 1
        el_replay = timed_region(args.steps, one, world, dist, sync)
    if D > 1 and args.pipeline and n_pol == 1:
        batch = capture_pipeline(torch, dev, pfb, pairs, inputs, C3_N_DAT, args.steps)
        el_pipe = timed_region(1, batch, world, dist, sync)
    # kernel-event region: the K steps eagerly with HIP events around every kernel (pair 0)
    lib.pfb_profile_reset()
    lib.pfb_profile_enable(1)
    timed_region(args.steps, steps[0], world, dist, sync)
    lib.pfb_profile_enable(0)
    kern = read_profile(lib, args.steps)
    lib.pfb_profile_reset()
    ms = el / args.steps * 1e3
    b_alg = 16.0 * (1.0 + 8.0 / 7.0) * C3_N_DAT * n_pol  # x in + chan out + chan in + output out
    gbs = b_alg / (ms * 1e-3) / 1e9
    K, n_out = pairs[0][2].shape[1], pairs[0][3].shape[1]
    res = {"workload": "C3 SKA-Mid padded round trip: 4096 ch, OS 8/7, %d two-stage firls taps, 2^26 "
                       "samples, Nf 512, Ov 128, tukey, deripple; 1 %s unit per step"
                       % (len(taps), "single-pol" if n_pol == 1 else "%d-pol" % n_pol),
           "n_pol": n_pol,
           "ms": round(ms, 4), "value": round(n_pol * C3_N_DAT / (ms * 1e-3) / 1e6, 2),
           "unit": "complex Msamples/s", "steps": args.steps,
           "ms_per_replay": round(el_replay / args.steps * 1e3, 4) if el_replay else None,
           "ms_pipelined": round(el_pipe / args.steps * 1e3, 4) if el_pipe else None,
           "plan_pairs": D, "pipeline": False, "hip_graph": "one graph of the K steps on one stream",
           "unit_seeds": [300 + 7919 * p for p in range(D)],
           "channelised_rows": K, "output_samples": n_out,
           "roofline": {"bound": "hbm", "alg_bytes_per_step": b_alg, "achieved": round(gbs, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4)},
           "kernels": kern}
    for ana, syn, _, _ in pairs:
        ana.close()
        syn.close()
    del pairs, inputs
    torch.cuda.empty_cache()
    return res


def measure_synthesis_only(args, torch, dist, world, dev, pfb, lib, ana, taps, x):
    """The standalone synthesis of a C2 channelised product resident in HBM —
    SynthesisPlan.execute(chan) = pfb_synthesis_execute: the channel IFFT (stage-1 rows)
    then the synthesis kernel; the PST production case, CBF-channelised input ->
    InverseFilterBank (InverseFilterBank.m:92-96, polyphase_synthesis.m:163-316)."""
    chan = ana.execute(x).contiguous()  # (n_pol, K, N) time-major, written by the analysis
    win = pfb.PFBWindow().lookup["tukey"](NF, OV)
    syn = pfb.SynthesisPlan(N_CHAN, OS_STR, NF, OV, True, 1, True, taps, win, None, chan.shape[0], dev.index or 0)
    K = chan.shape[1]
    n_out = syn.output_length(K)
    obuf = torch.empty((chan.shape[0], n_out), dtype=torch.complex64, device=dev)

    def step():
        syn.execute(chan, layout="ptc", out=obuf)
    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize(dev)
    sync = lambda: torch.cuda.synchronize(dev)  # noqa: E731
    # timed region: the K calls captured as one graph (no host launch gaps between the
    # calls' kernels); `ms_eager`: the K calls launched from Python one by one
    chain = capture_chain(torch, dev, [step] * args.steps)
    el = timed_region(1, chain, world, dist, sync)
    el_eager = timed_region(args.steps, step, world, dist, sync)
    lib.pfb_profile_reset()
    lib.pfb_profile_enable(1)
    timed_region(args.steps, step, world, dist, lambda: torch.cuda.synchronize(dev))
    lib.pfb_profile_enable(0)
    kern = read_profile(lib, args.steps)
    lib.pfb_profile_reset()
    ms = el / args.steps * 1e3
    n_pol = chan.shape[0]
    b_alg = 8.0 * n_pol * (K * N_CHAN + n_out)  # channelised product in + output out
    gbs = b_alg / (ms * 1e-3) / 1e9
    res = {"workload": "C2 synthesis only: (n_pol, %d, 256) channelised product of the C2 unit -> "
                       "%d output samples per pol (Nf 256, Ov 48, tukey, deripple)" % (K, n_out),
           "ms": round(ms, 4), "value": round(n_pol * n_out / (ms * 1e-3) / 1e6, 2),
           "unit": "complex Msamples/s (output samples)", "steps": args.steps,
           "ms_eager": round(el_eager / args.steps * 1e3, 4), "hip_graph": "one graph of the K calls",
           "roofline": {"bound": "hbm", "alg_bytes_per_step": b_alg, "achieved": round(gbs, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4)},
           "kernels": kern}
    del chan, obuf
    syn.close()
    return res


def run_device(args, torch, dist, world, rank, local, n_pol, n_dat, seeds, c3=None):
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    import ska_pst_dsp_model_amd as pfb
    from ska_pst_dsp_model_amd import _lib

    taps = pfb.design_PFB_FIR_filter(N_CHAN, OS_STR, TAPS_PER_CHAN)
    # independent units: one polarisation series per seed
    def units(sds):
        xs = []
        for sd in sds:
            g = torch.Generator(device=dev).manual_seed(sd)
            xs.append(torch.complex(torch.randn((n_dat,), device=dev, generator=g),
                                    torch.randn((n_dat,), device=dev, generator=g)) / np.sqrt(2.0))
        return torch.stack(xs).to(torch.complex64).contiguous()

    win = pfb.PFBWindow().lookup["tukey"](NF, OV)
    D = max(1, args.inflight)
    # pair 0 reads the rank's units (seeds above); with --distinct-inputs each further pair
    # reads its own units (seeds + 7919 p), so steps in flight never share input lines
    inputs = [units([sd + 7919 * p for sd in seeds]) if (p == 0 or args.distinct_inputs) else None
              for p in range(D)]
    inputs = [xi if xi is not None else inputs[0] for xi in inputs]
    x = inputs[0]
    pairs = []
    for _ in range(D):
        ana = pfb.AnalysisPlan(taps, N_CHAN, OS_STR, "polyphase_analysis", n_pol, local)
        syn = pfb.SynthesisPlan(N_CHAN, OS_STR, NF, OV, True, 1, True, taps, win, None, n_pol, local)
        if args.chunk_blocks:
            syn.set_chunk_blocks(args.chunk_blocks)
        syn.set_stage1_rows(args.stage1)
        K = ana.output_length(n_dat)
        n_out = syn.output_length(K)
        chan_buf = torch.empty((n_pol, K, N_CHAN), dtype=torch.complex64, device=dev)
        out_buf = torch.empty((n_pol, n_out), dtype=torch.complex64, device=dev)
        pairs.append((ana, syn, chan_buf, out_buf))
    ana, syn, chan_buf, out_buf = pairs[0]

    def make_step(ana, syn, chan_buf, out_buf, x):
        def step_serial():
            chan = ana.execute(x)            # (n_pol, K, N) time-major channelised data
            return syn.execute(chan, layout="ptc")

        def step_pipelined():
            return pfb.roundtrip(ana, syn, x, chan=chan_buf, out=out_buf)
        return step_pipelined if args.roundtrip else step_serial

    steps_of = [make_step(*p, inputs[i]) for i, p in enumerate(pairs)]
    step = steps_of[0]

    lib = _lib.load()
    if lib.pfb_build_flags() & 1:
        sys.exit(f"bench.py: {_lib.LIB_PATH} is an experiments build (A/B knobs, timing masks); "
                 f"benchmark the release library")
    # W untimed warm-up steps, dealt over the pairs like the timed ones (a pair that gets
    # none is still initialised by the eager call that precedes its graph capture)
    for i in range(args.warmup):
        steps_of[i % D]()
    torch.cuda.synchronize(dev)
    runs = list(steps_of)
    if args.graph:
        # the plans own all their device buffers after the warm-up, so the step is
        # capturable: one graph launch replays the step's kernels
        runs = [capture_step(torch, dev, s) for s in steps_of]
    if D == 1:
        run = runs[0]
    else:
        # step i on plan pair i mod D and stream i mod D: no dependence between the pairs
        # (each owns its buffers; the input is read-only), so the GPU may run one step's
        # analysis beside another's synthesis
        streams = [torch.cuda.Stream(device=dev) for _ in range(D)]
        ctr = [0]

        def run():
            i = ctr[0] % D
            ctr[0] += 1
            with torch.cuda.stream(streams[i]):
                runs[i]()

    def sync():
        torch.cuda.synchronize(dev)

    batch = None
    if args.pipeline and args.roundtrip and D > 1:
        # two-stream software pipeline over the K steps, captured as ONE graph
        batch = capture_pipeline(torch, dev, pfb, pairs, inputs, n_dat, args.steps)

    # timed region: K steps, no instrumentation (value, ms_per_step)
    if batch is not None:
        el = timed_region(1, batch, world, dist, sync)  # one replay = the K steps
    else:
        el = timed_region(args.steps, run, world, dist, sync)
    # the same K steps one at a time on one stream (pair 0, D = 1): ms_per_step_serial
    el_serial = el if D == 1 else timed_region(args.steps, runs[0], world, dist, sync)
    # profiled region: the same K steps with HIP events recorded around every kernel
    # launch on the library's launch stream (per-kernel durations for the roofline;
    # the events add inter-kernel gaps, so this region is not used for `value`).  The
    # kernels of a step run one after another on one stream, so a kernel's
    # event-bracketed duration is its own.
    lib.pfb_profile_reset()
    lib.pfb_profile_enable(args.kernel_events)
    el_prof = timed_region(args.steps, step, world, dist, sync)
    lib.pfb_profile_enable(0)

    # per-kernel-class event timings (on the library's launch stream)
    kern = read_profile(lib, args.steps)

    # A second reading of each kernel's duration: the step's halves (split round trip, pair 0)
    # launched K times back to back on torch's current stream — the library's launch stream —
    # between two HIP events (kernel + one dispatch gap, but consecutive analyses also queue
    # behind each other's write-back).  Reported beside the per-launch event pairs, which
    # feed `roofline`.
    if args.roundtrip and args.kernel_events and kern:
        a0, s0, c0, o0 = pairs[0]
        x0 = inputs[0]

        def batch_ms(fn):
            fn()
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.steps):
                fn()
            e1.record()
            torch.cuda.synchronize(dev)
            return e0.elapsed_time(e1) / args.steps
        try:
            t_a = batch_ms(lambda: pfb.roundtrip_analysis(a0, s0, x0, chan=c0))
            t_s = batch_ms(lambda: pfb.roundtrip_synthesis(a0, s0, n_dat, out=o0))
        except pfb.PfbError:
            t_a = t_s = None
        for key, t in (("analysis+chan_ifft", t_a), ("synth_block", t_s)):
            if t is not None and key in kern:
                kern[key]["back_to_back_avg_ms"] = t

    copy_gbs = copy_rate(torch, dev, lib) if rank == 0 else None

    e2e = None
    if args.e2e:
        e2e = e2e_pcie(torch, dev, pfb, ana, syn, n_pol, n_dat, chan_buf, out_buf, args.steps,
                       world, dist)
    # secondary keys of the N = 1 line (after the headline's regions; never its value)
    syn_only = c3_res = None
    if world == 1 and args.synthesis_only:
        syn_only = measure_synthesis_only(args, torch, dist, world, dev, pfb, lib, ana, taps, x)
    if world == 1 and c3 is not None:
        torch.cuda.synchronize(dev)
        torch.cuda.empty_cache()
        c3_res = measure_c3(args, torch, dist, world, dev, pfb, lib, c3)
        torch.cuda.synchronize(dev)
        torch.cuda.empty_cache()
        c3_res["dual_pol"] = measure_c3(args, torch, dist, world, dev, pfb, lib, c3, n_pol=2)
        if "cpu_baseline" in c3:
            c3_res["cpu_baseline"] = c3["cpu_baseline"]
    return {"el": el, "el_prof": el_prof, "el_serial": el_serial, "kern": kern, "copy_gbs": copy_gbs,
            "e2e": e2e, "taps": len(taps), "K": K, "n_out": n_out, "synthesis_only": syn_only,
            "c3": c3_res}


def report(args, res, world, workload, n_pol, n_dat, all_seeds):
    el, kern = res["el"], res["kern"]
    samples = world * n_pol * n_dat * args.steps
    value = samples / el / 1e6
    if kern:
        dom = max(kern, key=lambda k: kern[k]["avg_ms"] * kern[k]["launches"])
        kd = kern[dom]
        achieved = kd["alg_bytes_per_launch"] / (kd["avg_ms"] * 1e-3) / 1e9
    else:
        dom, achieved = None, 0.0
    kname = kern[dom].get("kernel") if dom else None
    traffic, why = traffic_for(workload, kname, pmc_traffic()) if dom else (None, "no kernel timed")
    if why and not args.stub_device:
        print(f"bench.py: WARNING roofline.traffic unavailable: {why}", file=sys.stderr, flush=True)
    roof = {"bound": "hbm", "kernel": kernel_key(kname) or dom, "kernel_class": dom,
            "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic}
    if why:
        roof["traffic_missing"] = why
    if res["copy_gbs"]:
        # the same achieved rate against the measured device-copy rate (not the peak)
        roof["copy_achievable"] = res["copy_gbs"]
        roof["frac_of_copy"] = round(achieved / res["copy_gbs"], 4)
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
        # the same K steps one at a time on one stream (no step in flight beside another)
        "ms_per_step_serial": round(res.get("el_serial", el) / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic CN(0,1) complex64 noise, HBM-resident, one torch generator seed per unit",
        "config": {"workload": WORKLOAD_NAMES[workload],
                   "n_chan": N_CHAN, "os_factor": OS_STR, "n_taps": res["taps"],
                   "n_dat_per_unit": n_dat, "n_pol_per_gpu": n_pol, "units": world * n_pol,
                   # every unit the timed region reads: step i runs pair i mod D, whose
                   # units are the rank's seeds + 7919 (i mod D) (--distinct-inputs)
                   "unit_seeds_per_rank": all_seeds,
                   "units_in_flight": len(all_seeds[0]) if all_seeds else n_pol,
                   "channelised_rows": res["K"], "output_samples_per_unit": res["n_out"],
                   "parallelism": f"{world} GPU(s) x {n_pol} independent unit(s), one process "
                                  f"per GPU, no collective on the data path",
                   "hip_graph": bool(args.graph),
                   "steps_in_flight": max(1, getattr(args, "inflight", 1)),
                   "pipeline": bool(getattr(args, "pipeline", 0)) and max(1, getattr(args, "inflight", 1)) > 1,
                   "distinct_inputs_per_pair": bool(getattr(args, "distinct_inputs", 1)),
                   "roundtrip_call": bool(args.roundtrip),
                   "stage1_rows": getattr(args, "stage1", "auto")},
        "roofline": roof,
        "round_trip_hbm_frac": round(rt_gbs / HBM_PEAK_GBS, 4),
        "ms_per_step_with_kernel_events": round(res["el_prof"] / args.steps * 1e3, 4),
        "kernels": kern,
    }
    traffic_all = pmc_traffic()

    def with_traffic(kc, wl):
        # PMC HBM bytes per launch of the same kernel in the same workload (pols included:
        # the records are keyed by workload, whose name fixes the pols per launch)
        kc["traffic"], _ = traffic_for(wl, kc.get("kernel"), traffic_all)
        if kc["traffic"] and kc.get("alg_bytes_per_launch"):
            kc["traffic_ratio"] = round(kc["traffic"] / kc["alg_bytes_per_launch"], 3)
            note = TRAFFIC_NOTES.get(kernel_key(kc.get("kernel")) or "")
            if kc["traffic_ratio"] > 1.6 and note:
                kc["traffic_note"] = note
    for kc in kern.values():  # PMC HBM bytes per launch of every timed kernel class
        with_traffic(kc, workload)
    for key in ("synthesis_only", "c3"):
        sec = res.get(key)
        if sec is None:
            continue
        wl = f"synthesis_only_p{n_pol}" if key == "synthesis_only" else key
        subs = [(sec, wl)] + ([(sec["dual_pol"], "c3_p2")] if key == "c3" and sec.get("dual_pol") else [])
        for ss, w in subs:
            for kc in ss.get("kernels", {}).values():
                with_traffic(kc, w)
                if kc["avg_ms"] > 0:
                    kc["achieved_GBs"] = round(kc["alg_bytes_per_launch"] / (kc["avg_ms"] * 1e-3) / 1e9, 1)
        out[key] = sec
    out["pfb_env"] = pfb_env()
    if args.stub_device:
        out["stub_device"] = True
    if res["e2e"] is not None:
        out["e2e_pcie"] = res["e2e"]
    return out


if __name__ == "__main__":
    main()
