#!/bin/bash
# Bench sweep on the GPU box: each line of SWEEP is "ENV_ASSIGNMENTS|BENCH_ARGS" (no profiler).
# Usage: TAG=x SWEEP=$'PBCCS_FILL_LANE=0|--steps 5\nPBCCS_FILL_LANE=1|--steps 10 --zmws-per-step 1000' bash tools/gpu_sweep2.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-sweep}
mkdir -p $OUT
i=0
while IFS='|' read -r envs args; do
  [ -z "$args$envs" ] && continue
  i=$((i+1))
  env $envs timeout -k 10 300 python -u bench.py --cpu-sample 0 --no-profile $args > $OUT/s_$i.json 2> $OUT/s_$i.err || { echo "run $i failed"; tail -20 $OUT/s_$i.err; exit 1; }
  echo "[$envs | $args] $(python3 -c "import json; d=json.load(open('$OUT/s_$i.json')); print(d['value'], d['config']['slots'], d['band_memory_gb'])")"
done <<< "$SWEEP"
