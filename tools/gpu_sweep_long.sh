#!/bin/bash
# GPU box: configs[2] (10 kb) through the work queue at several (slots, ZMWs per batch, HW queues) shapes.
# Usage: TAG=x N=480 SHAPES="5:0:16 16:15:32" bash tools/gpu_sweep_long.sh   (slots:batch:queues; batch 0 = planned)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-sweep}
mkdir -p $OUT
N=${N:-480}
WL=${WORKLOAD:-10kb}
for sh in ${SHAPES:-5:0:16}; do
  IFS=: read -r sl bz hq <<< "$sh"
  GPU_MAX_HW_QUEUES=$hq timeout -k 10 600 python -u bench.py --workload $WL --steps 8 --zmws-per-step $((N / 8)) --warmup 0 --cpu-sample 0 --streams $sl --batch-zmws $bz > $OUT/b_${sl}_${bz}_${hq}.json 2> $OUT/b_${sl}_${bz}_${hq}.err || { echo "bench $sh failed"; tail -20 $OUT/b_${sl}_${bz}_${hq}.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_${sl}_${bz}_${hq}.json')); print('$sh', d['value'], d['gcups'], d['zmw_status'], d['roofline']['in_flight'], d['band_memory_gb']['pool_mapped_bytes'])"
done
