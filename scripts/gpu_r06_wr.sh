#!/bin/bash
# Round 6: the streaming analysis FFT with wave barriers (WR) — bit-identity against the
# workgroup-barrier kernel (PFB_ANA_TV=8, experiments build), per-kernel A/B, the analysis /
# round-trip GPU tests on the release build, and bench.py with and without its CPU-baseline
# leg, interleaved (does the 25 s of all-core NumPy before the GPU regions move the GPU numbers?).
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd $R
EXP=$R/ska-pst-dsp-model_amd/lib/libpfb_hip_exp.so
: > gpurun_out/wr_digest.jsonl
for v in 0 8; do
  PFB_HIP_LIB=$EXP PFB_ANA_TV=$v timeout -k 10 200 python scripts/rt_digest.py --workload c2 --tag tv$v \
      >> gpurun_out/wr_digest.jsonl 2> gpurun_out/wr_digest.err || { tail -5 gpurun_out/wr_digest.err; exit 3; }
done
cat gpurun_out/wr_digest.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
    -k "analysis or roundtrip or round_trip or filterbank or stream or c2 or lowcbf or two_stage" > gpurun_out/pytest_wr.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_wr.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
ROUNDS=3 timeout -k 10 600 bash scripts/gpu_ab.sh wr:PFB_ANA_TV=0 wg:PFB_ANA_TV=8 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 4; }
cp gpurun_out/ab.jsonl gpurun_out/wr_ab.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/wr_ab.jsonl"):
    d = json.loads(l); print(d["tag"], {k: v["us"] for k, v in d.items() if isinstance(v, dict) and "us" in v})
PY
: > gpurun_out/cpu_order.jsonl
for i in 1 2; do
  for mode in cpu nocpu; do
    A=""; [ $mode = nocpu ] && A="--no-cpu-baseline"
    timeout -k 10 400 python bench.py --steps 20 --warmup 3 $A > gpurun_out/bench_$mode$i.json 2> gpurun_out/bench_$mode$i.err || exit 5
    python3 - $mode $i <<'PY' | tee -a gpurun_out/cpu_order.jsonl
import json, sys
d = json.load(open(f"gpurun_out/bench_{sys.argv[1]}{sys.argv[2]}.json"))
print(json.dumps({"mode": sys.argv[1], "round": int(sys.argv[2]), "value": d["value"], "ms_per_step": d["ms_per_step"],
                  "kernels_us": {k: round(v["avg_ms"] * 1e3, 1) for k, v in d["kernels"].items()},
                  "syn_only_ms": d["synthesis_only"]["ms"], "c3_ms": d["c3"]["ms"], "c3_ms_per_replay": d["c3"].get("ms_per_replay")}))
PY
  done
done
