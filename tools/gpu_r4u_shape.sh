#!/bin/bash
# one-off: batch shape at equal total work (40,000 configs[1] ZMWs): 5 slots x 2000-ZMW batches (the driver's shape)
# against more, smaller batches in flight
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4u; mkdir -p $OUT
for v in 5:2000:20 10:1000:40 8:1000:40 5:2000:20 10:1000:40 8:1000:40; do
  IFS=: read S Z K <<< "$v"
  timeout -k 10 300 python3 -u bench.py --streams $S --zmws-per-step $Z --steps $K --warmup 2 --cpu-sample 0 > $OUT/shape_${S}_${Z}.json 2> $OUT/shape.err || exit 1
  echo "slots=$S zmws=$Z steps=$K $(python3 -c "import json; d=json.load(open('$OUT/shape_${S}_${Z}.json')); print(d['value'], d['config'].get('slots'))")"
done
