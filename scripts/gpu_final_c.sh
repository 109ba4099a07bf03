#!/bin/bash
# The driver's bench command plain and under rocprofv3 (kernel trace + stats of the same
# command), then the C3 round trip one at a time vs pipelined over two streams.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_drv.json 2> gpurun_out/bench_drv.err || { tail -5 gpurun_out/bench_drv.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_drv.json')); print('C2', d['value'], d['ms_per_step'], json.dumps(d['roofline']), {k: round(v['avg_ms']*1e3,1) for k,v in d['kernels'].items()})"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_drv -o run \
    -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/prof_drv.log 2>&1
rc=$?; cd $R
if [ $rc -ne 0 ]; then echo "rocprof rc=$rc"; tail -5 gpurun_out/prof_drv.log; exit $rc; fi
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_drv/run_kernel_stats.csv')):
    if 'pfb' in r['Name']: print(r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us')
"
: > gpurun_out/c3_pipe.jsonl
for v in "1 0" "3 1" "1 0" "3 1"; do
  set -- $v
  timeout -k 10 240 python scripts/bench_aux.py --only-mid --inflight $1 --pipeline $2 >> gpurun_out/c3_pipe.jsonl 2> gpurun_out/c3.err || { tail -5 gpurun_out/c3.err; exit 1; }
done
cat gpurun_out/c3_pipe.jsonl
