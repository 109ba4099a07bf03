#!/bin/bash
# Per-kernel rocprofv3 kernel-trace stats of the C3 round trip for experiments-build variants
# ("tag" or "tag:ENV=V[,ENV=V]"): gpurun_out/c3k_<tag>/run_kernel_stats.csv.
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
for round in $(seq 1 ${ROUNDS:-1}); do
for v in "$@"; do
  tag=${v%%:*}; envs=""
  if [ "$tag" != "$v" ]; then envs=${v#*:}; envs=${envs//,/ }; fi
  rm -rf $R/gpurun_out/c3k_${tag}_$round
  env PFB_HIP_LIB=$R/ska-pst-dsp-model_amd/lib/libpfb_hip_exp.so $envs timeout -k 10 200 rocprofv3 --kernel-trace --stats \
      --output-format csv -d $R/gpurun_out/c3k_${tag}_$round -o run -- python3 $R/scripts/bench_aux.py --only-mid --reps 10 \
      > $R/gpurun_out/c3k_${tag}_$round.log 2>&1 || exit $?
  echo "== $tag round $round"
  python3 - $R/gpurun_out/c3k_${tag}_$round/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "pfb::" in r["Name"]:
        print(f'{float(r["AverageNs"])/1e3:8.1f} us x{r["Calls"]:>3} {r["Name"][:70]}')
PY
done
done
