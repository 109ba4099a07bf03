#!/bin/bash
# Round 6: the streaming analysis' channelised rows written as whole 1-KB runs from the
# wave-owned LDS rows — bit-identity against the direct 8-B stores (PFB_ANA_TV=32,
# experiments build), per-kernel A/B, the analysis-side GPU tests and the bench (release).
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd $R
EXP=$R/ska-pst-dsp-model_amd/lib/libpfb_hip_exp.so
: > gpurun_out/lines_digest.jsonl
for v in 0 32; do
  PFB_HIP_LIB=$EXP PFB_ANA_TV=$v timeout -k 10 200 python scripts/rt_digest.py --workload c2 --tag tv$v \
      >> gpurun_out/lines_digest.jsonl 2> gpurun_out/lines_digest.err || { tail -5 gpurun_out/lines_digest.err; exit 3; }
done
cat gpurun_out/lines_digest.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
    -k "analysis or roundtrip or round_trip or filterbank or stream or c2 or lowcbf or two_stage or sharding or smoke" > gpurun_out/pytest_lines.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_lines.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
ROUNDS=3 timeout -k 10 600 bash scripts/gpu_ab.sh lines:PFB_ANA_TV=0 direct:PFB_ANA_TV=32 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 4; }
cp gpurun_out/ab.jsonl gpurun_out/lines_ab.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/lines_ab.jsonl"):
    d = json.loads(l); print(d["tag"], {k: v["us"] for k, v in d.items() if isinstance(v, dict) and "us" in v})
PY
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_lines.json 2> gpurun_out/bench_lines.err || exit 5
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/bench_lines.json"))
print("C2", d["value"], d["ms_per_step"], "serial", d["ms_per_step_serial"], "frac", d["roofline"]["frac"], {k: round(v["avg_ms"] * 1e3, 1) for k, v in d["kernels"].items()})
print("syn_only", d["synthesis_only"]["ms"], "c3", d["c3"]["ms"], d["c3"].get("ms_per_replay"))
PY
