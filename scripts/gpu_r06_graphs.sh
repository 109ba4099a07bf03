#!/bin/bash
# Round 6: the C2 step as (1) bench.py's captured two-stream pipeline and (2) the same K steps
# captured in order on one stream as one graph (release build), interleaved, then the same
# under a rocprofv3 kernel trace (gpurun_out/prof_graphs_*).
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/graphs.jsonl
for round in 1 2 3; do
  for p in 1 2; do
    timeout -k 10 150 python scripts/inflight_ab.py --tag p$p --inflight 3 --pipeline $p --steps 20 --reps 5 \
        >> gpurun_out/graphs.jsonl 2> gpurun_out/graphs.err || { rc=$?; tail -5 gpurun_out/graphs.err; exit $rc; }
  done
done
cat gpurun_out/graphs.jsonl
export TMPDIR=/tmp
for p in 1 2; do
  rm -rf gpurun_out/prof_graphs_$p
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_graphs_$p -o run -- \
      python scripts/inflight_ab.py --tag p$p --inflight 3 --pipeline $p --steps 20 --reps 2 > gpurun_out/prof_graphs_$p.log 2>&1 || exit $?
done
