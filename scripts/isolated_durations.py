"""Per-kernel average duration of the launches in a rocprofv3 kernel trace that overlap no
other kernel of the library — bench.py's one-at-a-time region, which is what its in-dispatch
HIP events time (the pipelined region's launches overlap each other and run longer).

    python scripts/isolated_durations.py gpurun_out/prof_bench/bench_kernel_trace.csv
"""
import collections
import csv
import json
import sys


def main(path):
    rows = [r for r in csv.DictReader(open(path)) if "pfb::" in r["Kernel_Name"]]
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    acc = collections.defaultdict(list)
    for i, (s, e, n) in enumerate(iv):
        prev_end = max((iv[j][1] for j in range(max(0, i - 8), i)), default=0)
        nxt = iv[i + 1][0] if i + 1 < len(iv) else None
        if prev_end <= s and (nxt is None or nxt >= e):
            acc[n.split("(")[0].replace("void ", "")].append((e - s) / 1e3)
    out = {k: {"isolated_launches": len(v), "avg_us": round(sum(v) / len(v), 2)} for k, v in acc.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
