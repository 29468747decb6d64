#!/bin/bash
# Bench argument sweep on the GPU box (no profiler, no pytest). Usage: TAG=x ARGSETS="--a 1;--b 2" bash tools/gpu_sweep.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-sweep}
mkdir -p $OUT
i=0
IFS=';' read -ra AS <<< "${ARGSETS:-}"
for a in "${AS[@]}"; do
  i=$((i+1))
  echo "== args $i: $a"
  timeout -k 10 300 python -u bench.py --cpu-sample 0 $a > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { echo bench failed; tail -20 $OUT/bench_$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_$i.json')); print(d['value'], d['ms_per_step'], d['zmw_status'], d['roofline']['avg_launch_ms'])"
done
