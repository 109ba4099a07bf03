#!/bin/bash
# Round 6: the bench with the C3 and synthesis-only legs captured as one graph of the K steps
# (release build), the synthesis out= test, then the analysis timing variants (gpu_r06_tv.sh).
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf \
    -k "out_buffer or synthesis_baseline" > gpurun_out/pytest_chain.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_chain.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_chain.json 2> gpurun_out/bench_chain.err || exit 5
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/bench_chain.json"))
print("C2", d["value"], d["ms_per_step"], "frac", d["roofline"]["frac"])
so, c3 = d["synthesis_only"], d["c3"]
print("syn_only ms", so["ms"], "eager", so.get("ms_eager"), {k: round(v["avg_ms"] * 1e3, 1) for k, v in so["kernels"].items()})
print("c3 ms", c3["ms"], "per_replay", c3.get("ms_per_replay"), {k: round(v["avg_ms"] * 1e3, 1) for k, v in c3["kernels"].items()})
PY
bash scripts/gpu_r06_tv.sh
