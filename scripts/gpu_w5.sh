#!/bin/bash
# SKA-Mid wave synthesis (synth_wave512_kernel): its parity tests first (stop at the first
# failure), then the C3 round trip with the wave kernel (release) and the block kernel
# (experiments build, PFB_SYNTH_WAVE512=0), interleaved, and a kernel trace of the C3 round trip.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
PFB_PARITY_LOG=$R/gpurun_out/parity_w5.jsonl timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread -rf -k "nf512 or c3 or 4096 or baseline_shapes or roundtrip_matches or mid" \
    > gpurun_out/pytest_w5.log 2>&1
rc=$?; tail -8 gpurun_out/pytest_w5.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
: > gpurun_out/c3_w5.jsonl
for i in 1 2; do
  timeout -k 10 200 python scripts/bench_aux.py --only-mid >> gpurun_out/c3_w5.jsonl 2> gpurun_out/c3.err || { echo "c3 rel failed"; tail -5 gpurun_out/c3.err; exit 1; }
  PFB_HIP_LIB=$R/ska-pst-dsp-model_amd/lib/libpfb_hip_exp.so PFB_SYNTH_WAVE512=0 timeout -k 10 200 python scripts/bench_aux.py --only-mid >> gpurun_out/c3_w5.jsonl 2> gpurun_out/c3.err || { echo "c3 block failed"; tail -5 gpurun_out/c3.err; exit 1; }
done
cat gpurun_out/c3_w5.jsonl
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c3prof -o run \
    -- python3 $R/scripts/bench_aux.py --only-mid > $R/gpurun_out/c3prof.log 2>&1
rc=$?; cd $R
if [ $rc -ne 0 ]; then echo "rocprof rc=$rc"; tail -5 gpurun_out/c3prof.log; exit $rc; fi
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/c3prof/run_kernel_stats.csv')):
    if 'pfb' in r['Name']: print(r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us')
"
