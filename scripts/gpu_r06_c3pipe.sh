#!/bin/bash
# Round 6: C3 co-residency A/B — the SKA-Mid round trip one unit at a time vs the captured
# two-stream pipeline (unit i's FIR + row FFT beside unit i-1's synthesis), with the Nf-512
# synthesis held to 2 workgroups per CU by an LDS pad (PFB_W5_LDS_PAD, experiments build) so
# FIR / row-FFT workgroups can be resident beside it.  gpurun_out/c3pipe.jsonl
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
EXP=$GRAFT_REPO_ROOT/ska-pst-dsp-model_amd/lib/libpfb_hip_exp.so
C3V=${VARIANTS:-s:1:0 p:2:0 p:2:6400 p:3:6400 p:2:20000}
: > gpurun_out/c3pipe.jsonl
for round in $(seq 1 ${ROUNDS:-1}); do
for v in $C3V; do
  IFS=: read mode D pad <<< "$v"
  args="--only-mid --reps ${REPS:-6}"
  if [ "$mode" = p ]; then args="$args --inflight $D --pipeline 1 --graph 1"; fi
  out=$(env PFB_HIP_LIB=$EXP PFB_W5_LDS_PAD=$pad timeout -k 10 200 python scripts/bench_aux.py $args 2> gpurun_out/c3pipe.err) || { rc=$?; tail -5 gpurun_out/c3pipe.err; exit $rc; }
  echo "$out" | python3 -c "import sys,json; [print(json.dumps(dict(json.loads(l), variant='$v'))) for l in sys.stdin if l.startswith('{')]" | tee -a gpurun_out/c3pipe.jsonl
done
done
