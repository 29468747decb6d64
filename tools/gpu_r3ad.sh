#!/bin/bash
# GPU box: configs[2] (10 kb, 8 passes) at 2000 ZMWs through the work queue, slot count A/B (--streams).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3ad}
mkdir -p $OUT
run() {   # name, streams
  local name=$1 st=$2
  PBCCS_ROUND_TRACE=1 timeout -k 10 400 python -u bench.py --workload 10kb --steps 8 --zmws-per-step 250 --warmup 0 --cpu-sample 0 --streams $st > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -20 $OUT/$name.err; return 1; }
  echo "$name: $(python -c "import json; d=json.load(open('$OUT/$name.json')); print(d['value'], d['gcups'], d['zmw_status'], d['config'].get('slots'))")"
}
run s5 5 && run s8 8 && run s4 4
