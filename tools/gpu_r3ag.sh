#!/bin/bash
# GPU box: configs[3] (mixed) at 240 ZMWs on 5 / 8 / 12 slots, and configs[4] (SMRT-cell mix) on two
# self-launched ranks sharing cuda:0 (the multi-rank launch / dynamic queue / streamed gather rehearsal).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3ag}
mkdir -p $OUT
run() {   # name, args...
  local name=$1; shift
  timeout -k 10 500 python -u bench.py --cpu-sample 0 "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -20 $OUT/$name.err; return 1; }
  echo "$name: $(python -c "import json; d=json.load(open('$OUT/$name.json')); print(d['value'], d.get('gcups'), d.get('zmw_status'), d['n_gpus'], d['config'].get('slots'))")"
}
run mixed_s8 --workload mixed --steps 4 --zmws-per-step 60 --warmup 0 --streams 8 && \
run mixed_s12 --workload mixed --steps 4 --zmws-per-step 60 --warmup 0 --streams 12 && \
PBCCS_BENCH_DEVICE=0 run smrtcell_gpus2 --gpus 2 --workload smrtcell --steps 4 --zmws-per-step 60 --warmup 0 --streams 3
