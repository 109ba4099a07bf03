"""Practical HBM streaming rates on this box (the ceiling the HBM-bound kernels are judged
against beside the 8 TB/s datasheet figure): device-to-device copy (read + write), a
read-only reduction and a write-only fill, at the C3 stage sizes.  One JSON line per case.

    python scripts/hbm_probe.py > gpurun_out/hbm_probe.jsonl
"""
import json

import torch


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    dev = torch.device("cuda:0")
    for mb in (153, 306, 613, 1227):
        n = mb * (1 << 20) // 8
        src = torch.randn(n, dtype=torch.complex64, device=dev)
        dst = torch.empty_like(src)
        sf = torch.view_as_real(src).view(-1)
        for name, fn, nbytes in (
            ("copy", lambda: dst.copy_(src), 2 * n * 8),
            ("read_sum", lambda: sf.sum(), n * 8),
            ("write_fill", lambda: dst.fill_(0), n * 8),
        ):
            ms = timed(fn)
            print(json.dumps({"case": name, "MB_per_buffer": mb, "ms": round(ms, 4),
                              "GB/s": round(nbytes / ms / 1e6, 1)}), flush=True)
        del src, dst, sf
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
