"""Account for every microsecond of the C3 round-trip step in a rocprofv3 kernel trace of
bench.py: the C3 kernels (FIR -> row FFT -> Nf-512 synthesis, plus anything else the library
launches between them) are cut into segments at host gaps > 1 ms (warmup, the timed graph
replays, the kernel-event region); per segment: steps, step period (first kernel start to the
next step's first kernel start), each kernel's average duration and the average idle gap
after it.

    python scripts/c3_step_trace.py gpurun_out/prof_c3/run_kernel_trace.csv
"""
import csv
import json
import statistics
import sys

C3_KERNELS = ("fir_lds_kernel", "row_fft4096", "synth_wave512")


def short(name):
    return name.split("(")[0].replace("void ", "").replace("pfb::", "")


def main(path):
    rows = [r for r in csv.DictReader(open(path)) if "pfb::" in r["Kernel_Name"]]
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
    # the C3 part of the trace: from the first C3 FIR launch on, up to the last C3 synthesis
    first = next(i for i, k in enumerate(iv) if k[2].startswith(C3_KERNELS[0]))
    last = max(i for i, k in enumerate(iv) if k[2].startswith(C3_KERNELS[2]))
    iv = iv[first:last + 1]
    segs, cur = [], [iv[0]]
    for k in iv[1:]:
        if k[0] - cur[-1][1] > 1_000_000:
            segs.append(cur)
            cur = []
        cur.append(k)
    segs.append(cur)
    out = []
    for s in segs:
        starts = [k[0] for k in s if k[2].startswith(C3_KERNELS[0])]
        n = len(starts)
        per = {}
        for i, k in enumerate(s):
            gap = (s[i + 1][0] - k[1]) / 1e3 if i + 1 < len(s) else None
            d = per.setdefault(k[2][:60], {"dur": [], "gap_after": []})
            d["dur"].append((k[1] - k[0]) / 1e3)
            if gap is not None:
                d["gap_after"].append(gap)
        period = [(b - a) / 1e3 for a, b in zip(starts, starts[1:])]
        out.append({
            "steps": n,
            "span_us": round((s[-1][1] - s[0][0]) / 1e3, 1),
            "step_period_us": round(statistics.mean(period), 1) if period else None,
            "kernels": {k: {"launches": len(v["dur"]), "avg_us": round(statistics.mean(v["dur"]), 1),
                            "avg_gap_after_us": round(statistics.mean(v["gap_after"]), 2) if v["gap_after"] else None}
                        for k, v in per.items()},
        })
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
