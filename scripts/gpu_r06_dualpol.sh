#!/bin/bash
# Round 6: the SKA-Mid dual-pol unit — its GPU test, the bench line (c3.dual_pol) and its PMC
# traffic record (c3_p2).
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
    -k "dual_pol or c3_parameters or out_buffer" > gpurun_out/pytest_dual.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_dual.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
WORKLOADS=c3p2 timeout -k 10 300 bash scripts/gpu_pmc_r06.sh > gpurun_out/pmc_dual.log 2>&1 || { tail -5 gpurun_out/pmc_dual.log; exit 4; }
cp gpurun_out/pmc_traffic.json gpurun_out/pmc_traffic_c3p2.json
tail -4 gpurun_out/pmc_dual.log
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_dual.json 2> gpurun_out/bench_dual.err || exit 5
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/bench_dual.json"))
print("C2", d["value"], d["ms_per_step"])
c3 = d["c3"]; dp = c3["dual_pol"]
print("c3", c3["ms"], "dual", dp["ms"], dp["value"], dp["roofline"]["frac"], {k: round(v["avg_ms"] * 1e3, 1) for k, v in dp["kernels"].items()})
PY
