"""CPU tests of bench.py's multi-GPU entry point (BASELINE C4 sharding).

``bench.py --gpus N`` starts N ranks itself through torch.distributed.run (a child
process; the parent makes no GPU call), each rank owns its units (one dual-pol DADA
time block = 2 units, seeds 100+2r, 100+2r+1) and rank 0 reports
value = all ranks' samples / max-over-ranks time.  Here the device step is stubbed
(``--stub-device``: a fixed CPU wait, gloo backend), so the launcher, the unit mapping
and the aggregation run on the CPU.
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def test_rank_units_cover_c4_seeds_once():
    seeds = [s for r in range(8) for s in bench.rank_units("c4", r)]
    assert seeds == list(range(100, 116))  # 16 units, 2 per GPU on 8 GPUs
    assert bench.rank_units("c2", 0) == [100]
    assert bench.rank_units("c4", 3) == [106, 107]


def test_workload_defaults():
    class A:
        workload = "auto"
    assert bench.resolve_workload(A, 1) == "c2"
    assert bench.resolve_workload(A, 2) == "c4"
    A.workload = "c4"
    assert bench.resolve_workload(A, 1) == "c4"


def _run(args, env=None, timeout=240):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=e,
                          capture_output=True, text=True, timeout=timeout, cwd=REPO)


def _json_line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_gpus_2_launches_two_ranks_and_aggregates():
    steps = 4
    r = _run(["--gpus", "2", "--stub-device", "--steps", str(steps), "--warmup", "1",
              "--no-cpu-baseline"])
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    cfg = d["config"]
    assert cfg["workload"].startswith("C4")
    assert cfg["n_pol_per_gpu"] == 2 and cfg["units"] == 4
    # 3 steps in flight (default), each plan pair on its own units (seeds + 7919 p)
    assert cfg["unit_seeds_per_rank"] == [[100, 101, 8019, 8020, 15938, 15939],
                                          [102, 103, 8021, 8022, 15940, 15941]]
    assert cfg["units_in_flight"] == 6
    # value = all ranks' samples / max-over-ranks time
    samples = 2 * 2 * cfg["n_dat_per_unit"] * steps
    t = d["ms_per_step"] * steps / 1e3
    assert abs(d["value"] - samples / t / 1e6) / d["value"] < 1e-3
    assert d["cpu_baseline"] is None  # the CPU leg runs at N = 1 only


def test_gpus_1_is_the_c2_headline():
    r = _run(["--stub-device", "--steps", "2", "--warmup", "0", "--no-cpu-baseline"])
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 1
    assert d["config"]["workload"].startswith("C2")
    assert d["config"]["unit_seeds_per_rank"] == [[100, 8019, 15938]]
    assert d["config"]["units_in_flight"] == 3
    assert d["ms_per_step_serial"] > 0
    r = _run(["--stub-device", "--steps", "2", "--warmup", "0", "--no-cpu-baseline",
              "--inflight", "1"])
    d = _json_line(r.stdout)
    assert d["config"]["unit_seeds_per_rank"] == [[100]] and d["config"]["units_in_flight"] == 1


def test_gpus_must_match_launcher_world():
    r = _run(["--gpus", "2", "--stub-device", "--no-cpu-baseline"],
             env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in (r.stderr + r.stdout)


def test_refuses_work_dropping_knobs():
    """A PFB_* knob (here a timing mask that drops the kernels' loads in an experiments
    build) makes the bench exit non-zero before anything is timed."""
    r = _run(["--stub-device", "--no-cpu-baseline", "--steps", "1", "--warmup", "0"],
             env={"PFB_TIMING_MASK": "1"})
    assert r.returncode != 0
    assert "PFB_TIMING_MASK" in (r.stderr + r.stdout)


def test_env_is_recorded():
    r = _run(["--stub-device", "--no-cpu-baseline", "--steps", "1", "--warmup", "0"],
             env={"PFB_PARITY_LOG": "/dev/null"})
    assert r.returncode == 0, r.stderr[-3000:]
    assert _json_line(r.stdout)["pfb_env"] == {"PFB_PARITY_LOG": "/dev/null"}


def _report(workload, kernels, n_pol):
    class A:
        steps, warmup, graph, roundtrip, stub_device = 10, 3, 1, 1, True
    res = {"el": 1e-3, "el_prof": 1e-3, "el_serial": 1.5e-3, "kern": kernels, "copy_gbs": None,
           "e2e": None, "taps": 3073, "K": 74883, "n_out": 16737280}
    return bench.report(A, res, 1, workload, n_pol, 1 << 24, [[100]])


def test_roofline_traffic_is_the_pmc_record_of_the_timed_kernel():
    """roofline.traffic = the committed PMC bytes of the kernel the library names for the
    dominant class (matched by kernel name, not by class), else null with the reason."""
    traffic = bench.pmc_traffic()
    assert "c2" in traffic and traffic["c2"], "profiles/pmc_traffic.json has no C2 records"
    name, rec = max(traffic["c2"].items(), key=lambda kv: kv[1]["bytes"])
    kern = {"analysis+chan_ifft": {"kernel": f"void pfb::{name}(pfb::AnalysisArgs)", "avg_ms": 0.09,
                                   "launches": 10, "alg_bytes_per_launch": 2.8e8, "ms_per_step": 0.09},
            "synth_block": {"kernel": "void pfb::other_kernel<1>(pfb::SynthBlockArgs)", "avg_ms": 0.05,
                            "launches": 10, "alg_bytes_per_launch": 2.8e8, "ms_per_step": 0.05}}
    roof = _report("c2", kern, 1)["roofline"]
    assert roof["kernel"] == name and roof["traffic"] == rec["bytes"]
    assert "traffic_missing" not in roof
    # a kernel without a PMC record: null, and the reason is in the line
    kern["analysis+chan_ifft"]["kernel"] = "void pfb::not_profiled<2>(pfb::AnalysisArgs)"
    roof = _report("c2", kern, 1)["roofline"]
    assert roof["traffic"] is None and "not_profiled<2>" in roof["traffic_missing"]


def test_report_states_what_was_timed():
    """The line lists every unit seed the timed region reads, the units in flight, and the
    one-at-a-time step time beside the pipelined one."""
    out = _report("c2", {}, 1)
    assert out["ms_per_step"] == 0.1 and out["ms_per_step_serial"] == 0.15
    seeds = bench.pair_seeds([100], 3, True)
    assert seeds == [100, 8019, 15938]
    assert bench.pair_seeds([100, 101], 2, False) == [100, 101, 100, 101]
    class A:
        steps, warmup, graph, roundtrip, stub_device, inflight = 10, 3, 1, 1, True, 3
    res = {"el": 1e-3, "el_prof": 1e-3, "el_serial": 1.7e-3, "kern": {}, "copy_gbs": None,
           "e2e": None, "taps": 3073, "K": 74883, "n_out": 16737280}
    out = bench.report(A, res, 1, "c2", 1, 1 << 24, [seeds])
    assert out["config"]["unit_seeds_per_rank"] == [[100, 8019, 15938]]
    assert out["config"]["units_in_flight"] == 3
    assert out["ms_per_step_serial"] == 0.17
