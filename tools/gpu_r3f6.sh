#!/bin/bash
# GPU box, long-template and multi-rank lines at HEAD: configs[2] at 2000 ZMWs, configs[3] mixed-240, and the
# two-rank SMRT-cell rehearsal on one device (default slots each).  Each GPU step has its own limit.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3f6}
mkdir -p $OUT
run() {   # name, args...
  local name=$1; shift
  timeout -k 10 400 python -u bench.py --cpu-sample 0 "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -20 $OUT/$name.err; return 1; }
  echo "$name: $(python -c "import json; d=json.load(open('$OUT/$name.json')); print(d['value'], d.get('gcups'), d.get('zmw_status'), d['n_gpus'], d['config'].get('slots'))")"
}
run b10_2000 --workload 10kb --steps 8 --zmws-per-step 250 --warmup 0 && \
run mixed240 --workload mixed --steps 4 --zmws-per-step 60 --warmup 0 && \
PBCCS_BENCH_DEVICE=0 run smrtcell_gpus2 --gpus 2 --workload smrtcell --steps 4 --zmws-per-step 60 --warmup 0 --streams 3
