#!/bin/bash
# one-off: more slots of 1000-ZMW batches with 32 hardware queues (two streams per slot) against 8 slots on 16 queues
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4x; mkdir -p $OUT
for v in 8:16 10:32 12:32 8:16 10:32 12:32; do
  S=${v%:*}; Q=${v#*:}
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python3 -u bench.py --steps 24 --warmup 2 --cpu-sample 0 --streams $S > $OUT/q_${S}_${Q}.json 2> $OUT/q.err || exit 1
  echo "slots=$S queues=$Q $(python3 -c "import json; d=json.load(open('$OUT/q_${S}_${Q}.json')); print(d['value'], d['config']['slots'])")"
done
