"""The BASELINE configs[4] purity sweep (current_performance.m temporal impulses and
tones + the sgcht.m frequency comb and square wave; sub-config 'mid') on the HIP engine,
scored as the reference scores it (verify.score_vector).  One JSON record per vector,
then a summary line.

    python scripts/purity_sweep.py [--npoints 300] [--batch 16]
    python -m torch.distributed.run --nproc-per-node 8 scripts/purity_sweep.py ...

Under a launcher the vectors are dealt round-robin over the ranks (one GPU each, no
collective on the data path); every rank writes its records to --out-dir and rank 0
merges them after a gloo barrier."""
import argparse
import glob
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ska-pst-dsp-model_amd"), REPO]


def summary(recs, seconds, world):
    imp = [r for r in recs if r["domain"] == "time" and "expected_index" in r]
    ton = [r for r in recs if r["domain"] == "freq"]
    return {"summary": True, "vectors": len(recs), "gpus": world,
            "impulses_in_output": len(imp),
            "impulses_at_expected_index": sum(r["peak_index"] == r["expected_index"] for r in imp),
            "worst_impulse_outside_pm1_dB": max((r["max_outside_pm1_dB"] for r in imp), default=None),
            "worst_impulse_max_spurious_dB_pm30": max((r["max_spurious_dB"] for r in imp), default=None),
            "tones": len(ton),
            "worst_tone_max_spurious_dB": max((r["max_spurious_dB"] for r in ton), default=None),
            "worst_tone_total_spurious_dB": max((r["total_spurious_dB"] for r in ton), default=None),
            "worst_tone_max_diff_dB": max((r["max_diff_dB"] for r in ton), default=None),
            "comb_test": [r["comb_test"] for r in recs if r["domain"] == "comb"],
            "square_wave": [{k: r[k] for k in ("on_power", "off_power")}
                            for r in recs if r["domain"] == "square_wave"],
            "seconds": round(seconds, 1)}


def stub_sweep(verify, npoints, rank, world, max_vectors=0):
    """The sweep's vector list and round-robin share (verify.purity_sweep's, 'mid'
    alignment), each vector 'scored' with fixed synthetic numbers that name its rank."""
    al = verify.performance_alignment(4096, "8/7", 512, 128, 100353, 3, 0, 0)
    items = verify.sweep_vectors(al, npoints, 3) + [("comb", 32), ("square_wave", 3981)]
    if max_vectors:
        items = items[:max_vectors]
    recs = []
    for kind, p in verify.shard(items, rank, world):
        r = {"domain": kind, "param": p, "rank": rank}
        if kind == "time":
            r.update(peak_index=p, expected_index=p, max_outside_pm1_dB=-80.0, max_spurious_dB=-90.0)
        elif kind == "freq":
            r.update(max_spurious_dB=-70.0, total_spurious_dB=-65.0, max_diff_dB=-100.0)
        elif kind == "comb":
            r.update(comb_test=0)
        else:
            r.update(on_power=1.0, off_power=0.0)
        recs.append(r)
    return recs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--npoints", type=int, default=300)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--max-vectors", type=int, default=0)
    ap.add_argument("--out-dir", default=os.path.join(REPO, "gpurun_out", "purity"))
    ap.add_argument("--stub", action="store_true",
                    help="test hook: score nothing on a device; each rank emits one synthetic "
                         "record per vector of its round-robin share (exercises the sharding "
                         "and the rank-file merge on the CPU)")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    from ska_pst_dsp_model_amd import verify
    t0 = time.perf_counter()
    if args.stub:
        recs = stub_sweep(verify, args.npoints, rank, world, args.max_vectors)
    else:
        recs = verify.purity_sweep(device=local, npoints=args.npoints, batch=args.batch, rank=rank,
                                   world=world, max_vectors=args.max_vectors)
    if world == 1:
        for r in recs:
            print(json.dumps(r), flush=True)
        print(json.dumps(summary(recs, time.perf_counter() - t0, world)), flush=True)
        return
    import torch.distributed as dist
    os.makedirs(args.out_dir, exist_ok=True)
    with open(os.path.join(args.out_dir, f"rank{rank}.jsonl"), "w") as f:
        for r in recs:
            f.write(json.dumps(r) + "\n")
    dist.init_process_group("gloo")
    dist.barrier()
    if rank == 0:
        allr = []
        for p in sorted(glob.glob(os.path.join(args.out_dir, "rank*.jsonl"))):
            with open(p) as f:
                allr += [json.loads(line) for line in f]
        for r in allr:
            print(json.dumps(r), flush=True)
        print(json.dumps(summary(allr, time.perf_counter() - t0, world)), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
