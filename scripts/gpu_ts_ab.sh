#!/bin/bash
# TwoStage cascade A/B over the experiments library's launch knobs: ROUNDS interleaved
# rounds of bench_aux.py --only-twostage per tag ("tag:ENV=V[,ENV=V]" arguments).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/ts_ab.jsonl
for round in $(seq 1 ${ROUNDS:-2}); do
  for spec in "$@"; do
    tag=${spec%%:*}; envs=${spec#*:}; [ "$envs" = "$spec" ] && envs=""
    env $(echo "$envs" | tr ',' ' ') PFB_HIP_LIB=ska-pst-dsp-model_amd/lib/libpfb_hip_exp.so \
      timeout -k 10 120 python scripts/bench_aux.py --only-twostage --reps 20 2>> gpurun_out/ts_ab.err \
      | grep "stream call" | sed "s/^{/{\"tag\": \"$tag\", \"round\": $round, /" >> gpurun_out/ts_ab.jsonl || exit $?
  done
done
python3 -c "
import json
for l in open('gpurun_out/ts_ab.jsonl'):
    d = json.loads(l); print(d['tag'], d['round'], d['ms'])
"
