"""The BASELINE configs[4] purity sweep (temporal impulses, tones, frequency comb, square
wave; SKA-Mid padded parameters) on one GPU: prints one JSON record per test vector and a
summary line.  Usage: python scripts/purity_sweep.py [--npoints N] [--batch B]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ska-pst-dsp-model_amd"), REPO]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--npoints", type=int, default=16)
    ap.add_argument("--batch", type=int, default=8)
    args = ap.parse_args()
    from ska_pst_dsp_model_amd import verify
    t0 = time.perf_counter()
    recs = verify.purity_sweep(npoints=args.npoints, batch=args.batch)
    for r in recs:
        print(json.dumps(r), flush=True)
    imp = [r for r in recs if r["kind"] == "impulse"]
    ton = [r for r in recs if r["kind"] == "tone"]
    print(json.dumps({"summary": True, "vectors": len(recs),
                      "worst_impulse_max_spurious_dB": max(r["max_spurious"] for r in imp),
                      "worst_tone_max_spurious_dB": max(r["max_spurious"] for r in ton),
                      "comb_test": [r["comb_test"] for r in recs if r["kind"] == "comb"],
                      "seconds": round(time.perf_counter() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
