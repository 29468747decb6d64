#!/bin/bash
# one-off: the driver's command with the new batch shape (8 slots x 1000-ZMW batches) against the round-3 shape
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4w; mkdir -p $OUT
for v in new old new old; do
  A=""; [ $v = old ] && A="--streams 5 --batch-split 1"
  timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 $A > $OUT/drv_$v.json 2> $OUT/drv_$v.err || exit 1
  echo "$v $(python3 -c "import json; d=json.load(open('$OUT/drv_$v.json')); print(d['value'], d['config']['slots'], d['config'].get('device_batch_zmws'))")"
done
