#!/bin/bash
# HBM traffic of the fill kernels: two PMC passes (FETCH_SIZE, WRITE_SIZE; they do not fit one pass)
# over the default bench command, then tools/pmc_traffic.py.  Usage: TAG=x bash tools/gpu_traffic.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-traffic}
mkdir -p $OUT
ARGS="--cpu-sample 0 ${BENCH_ARGS}"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/fetch -o pmc -- python3 -u bench.py $ARGS > $OUT/fetch.json 2> $OUT/fetch.err || { echo "fetch pass failed"; tail -5 $OUT/fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/write -o pmc -- python3 -u bench.py $ARGS > $OUT/write.json 2> $OUT/write.err || { echo "write pass failed"; tail -5 $OUT/write.err; exit 1; }
F=$(find $OUT/fetch -name "*counter_collection.csv" | head -1)
W=$(find $OUT/write -name "*counter_collection.csv" | head -1)
for k in k_fill_tall k_fill k_score; do
  python3 tools/pmc_traffic.py "$F" "$W" $OUT/fetch.json $OUT/traffic_${k#k_}.json $k > /dev/null || echo "no $k dispatches"
done
cat $OUT/traffic_fill_tall.json
gzip -f "$F" "$W"
