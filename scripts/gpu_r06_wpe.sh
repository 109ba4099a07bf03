#!/bin/bash
# Round 6: the C2 streaming analysis at 3 waves per SIMD (PFB_ANA_WPE=3, experiments build)
# against the release shape (184 VGPRs, 2 per SIMD), bit-identity of its round trip, and a
# kernel trace of bench.py (release build) whose C3 part scripts/c3_step_trace.py accounts for.
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd $R
EXP=$R/ska-pst-dsp-model_amd/lib/libpfb_hip_exp.so
: > gpurun_out/wpe_digest.jsonl
for v in 0 3; do
  PFB_HIP_LIB=$EXP PFB_ANA_WPE=$v timeout -k 10 200 python scripts/rt_digest.py --workload c2 --tag wpe$v \
      >> gpurun_out/wpe_digest.jsonl 2> gpurun_out/wpe_digest.err || { tail -5 gpurun_out/wpe_digest.err; exit 3; }
done
cat gpurun_out/wpe_digest.jsonl
ROUNDS=3 timeout -k 10 900 bash scripts/gpu_ab.sh wpe2:PFB_ANA_WPE=0 wpe3:PFB_ANA_WPE=3 wpe3c2:PFB_ANA_WPE=3,PFB_ANA_WG_PER_CU=2 \
    wpe2c3:PFB_ANA_WG_PER_CU=3 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 4; }
cp gpurun_out/ab.jsonl gpurun_out/wpe_ab.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/wpe_ab.jsonl"):
    d = json.loads(l); print(d["tag"], {k: v["us"] for k, v in d.items() if isinstance(v, dict) and "us" in v})
PY
cd /tmp
rm -rf $R/gpurun_out/prof_trace
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_trace -o run -- \
    python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/bench_trace.json 2> $R/gpurun_out/bench_trace.err || exit 5
cd $R
python3 scripts/c3_step_trace.py gpurun_out/prof_trace/run_kernel_trace.csv > gpurun_out/c3_step_trace.json
cat gpurun_out/c3_step_trace.json
