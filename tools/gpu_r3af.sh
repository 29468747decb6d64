#!/bin/bash
# GPU box: tools/gpu_r3ae.sh (Quiver arena pre-size A/B + traffic at the working tree), then configs[2] at 2000
# ZMWs with 10 and 12 slots.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TAG=r3ae bash tools/gpu_r3ae.sh || exit 1
OUT=gpurun_out/r3af
mkdir -p $OUT
run() {   # name, streams
  local name=$1 st=$2
  timeout -k 10 400 python -u bench.py --workload 10kb --steps 8 --zmws-per-step 250 --warmup 0 --cpu-sample 0 --streams $st > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -20 $OUT/$name.err; return 1; }
  echo "$name: $(python -c "import json; d=json.load(open('$OUT/$name.json')); print(d['value'], d['gcups'], d['zmw_status'], d['config'].get('slots'))")"
}
run s10 10 && run s12 12 && run s8 8
