"""Probe: does an intermediate that is written and read back in Infinity-Cache-sized chunks
cost less than one written and read back whole?  (Design question for the C3 round trip,
DESIGN.md §11: the FIR's stage-1 rows Z are written once and read twice.)

  whole:    Z = x (copy, 614 MB), out = Z (copy)              -- Z round-trips HBM
  chunked:  for each chunk c: Zc = x[c]; out[c] = Zc           -- Zc (S MB) reused, L3-resident

Prints one JSON line per (mode, chunk MB): ms (median of reps) and the HBM-equivalent rate.
"""
import json
import sys

import torch


def main():
    dev = torch.device("cuda", 0)
    n = 614 * (1 << 20) // 4  # float32 elements of a C3-sized Z (614 MB)
    x = torch.ones(n, device=dev)
    out = torch.empty_like(x)
    reps = 10

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        return ts[len(ts) // 2]

    z = torch.empty_like(x)

    def whole():
        z.copy_(x)
        out.copy_(z)
    ms = timeit(whole)
    print(json.dumps({"mode": "whole", "ms": round(ms, 4), "bytes": 4 * n * 4,
                      "TBps_if_all_hbm": round(4 * n * 4 / ms / 1e9, 2)}), flush=True)
    for mb in (16, 32, 64, 128, 192):
        m = mb * (1 << 20) // 4
        zc = torch.empty(m, device=dev)
        chunks = [(i, min(i + m, n)) for i in range(0, n, m)]

        def chunked():
            for a, b in chunks:
                zc[:b - a].copy_(x[a:b])
                out[a:b].copy_(zc[:b - a])
        ms = timeit(chunked)
        print(json.dumps({"mode": "chunked", "chunk_MB": mb, "chunks": len(chunks), "ms": round(ms, 4),
                          "TBps_if_all_hbm": round(4 * n * 4 / ms / 1e9, 2)}), flush=True)
    # the read-twice case (FIR writes Z, row FFT reads it, synthesis reads it again)
    def whole3():
        z.copy_(x)
        out.copy_(z)
        out.add_(z)
    ms = timeit(whole3)
    print(json.dumps({"mode": "whole_read_twice", "ms": round(ms, 4)}), flush=True)
    for mb in (32, 64, 128):
        m = mb * (1 << 20) // 4
        zc = torch.empty(m, device=dev)
        chunks = [(i, min(i + m, n)) for i in range(0, n, m)]

        def chunked3():
            for a, b in chunks:
                zc[:b - a].copy_(x[a:b])
                out[a:b].copy_(zc[:b - a])
                out[a:b].add_(zc[:b - a])
        ms = timeit(chunked3)
        print(json.dumps({"mode": "chunked_read_twice", "chunk_MB": mb, "ms": round(ms, 4)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
