"""Summarise rocprofv3 --pmc CSV passes per kernel (mean counter value per dispatch).

HBM traffic follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read, so read bytes =
2 * FETCH_SIZE * 1024 (the guide's correction); WRITE_SIZE * 1024 is exact for 16-B
streaming stores.  Infinity-Cache hits are counted too (the counters sit on the L2's
memory side), so this is L2<->fabric traffic, an upper bound of HBM traffic.
"""
import collections
import csv
import glob
import json
import sys


def short(name):
    for k in ("analysis_fused", "analysis_stream", "row_fft", "synth_block", "synth_wave", "fir_generic", "fir_window",
              "fir_lds", "spectral", "tile_transpose"):
        if k in name:
            return name.split("(")[0].replace("void pfb::", "")
    return None


def load(dirs):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = short(row["Kernel_Name"])
                    if k:
                        acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def traffic_json(res):
    """Per kernel (bench.py's kernel_key form): HBM bytes per launch
    (2 x FETCH_SIZE KiB + WRITE_SIZE KiB)."""
    out = {}
    for k, cs in res.items():
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        rd = 2 * cs["FETCH_SIZE"] * 1024
        wr = cs["WRITE_SIZE"] * 1024
        out[k] = {"read_bytes": rd, "write_bytes": wr, "bytes": rd + wr}
    return out


if __name__ == "__main__":
    args = sys.argv[1:]
    js = None
    if args and args[0] == "--json":
        # --json OUT WORKLOAD DIR...: merge this workload's records into OUT (bench.py
        # looks the timed kernel up as OUT[workload][kernel])
        js, workload, args = args[1], args[2], args[3:]
    res = load(args if args else ["."])
    if js:
        try:
            with open(js) as f:
                doc = json.load(f)
        except (OSError, ValueError):
            doc = {}
        doc[workload] = traffic_json(res)
        with open(js, "w") as f:
            json.dump(doc, f, indent=1, sort_keys=True)
    for k, cs in res.items():
        print(f"== {k}")
        for c in sorted(cs):
            print(f"   {c:28s} {cs[c]:16.1f}")
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            rd = 2 * cs["FETCH_SIZE"] * 1024
            wr = cs["WRITE_SIZE"] * 1024
            print(f"   -> read {rd/1e6:.1f} MB (2x FETCH_SIZE), write {wr/1e6:.1f} MB per dispatch")
        if "SQ_LDS_BANK_CONFLICT" in cs and "SQ_LDS_IDX_ACTIVE" in cs:
            print(f"   -> LDS bank-conflict cycles / LDS active = "
                  f"{cs['SQ_LDS_BANK_CONFLICT']/max(cs['SQ_LDS_IDX_ACTIVE'],1):.3f}")
        if "SQ_WAVE_CYCLES" in cs:
            w = cs["SQ_WAVE_CYCLES"]
            print(f"   -> wait_any {cs.get('SQ_WAIT_ANY',0)/w:.2f}  wait_inst {cs.get('SQ_WAIT_INST_ANY',0)/w:.2f}"
                  f"  active {cs.get('SQ_ACTIVE_INST_ANY',0)/w:.2f} of wave cycles")
