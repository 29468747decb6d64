#!/bin/bash
# GPU box: interleaved bench runs of several in-tree library builds (PBCCS_LIB), ROUNDS times each.
# Usage: TAG=x LIBS="a.so b.so" ROUNDS=2 bash tools/gpu_libs.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-libs}
mkdir -p $OUT
for i in $(seq 1 ${ROUNDS:-2}); do
  for l in $LIBS; do
    n=$(basename $l .so)
    PBCCS_LIB=$GRAFT_REPO_ROOT/pbccs_amd/_lib/$l timeout -k 10 300 python -u bench.py --cpu-sample 0 --no-profile ${BENCH_ARGS} > $OUT/${n}_$i.json 2> $OUT/${n}_$i.err || { echo "bench $n failed"; tail -20 $OUT/${n}_$i.err; exit 1; }
    echo "$n: $(python -c "import json; d=json.load(open('$OUT/${n}_$i.json')); print(d['value'], d['zmw_status'])")"
  done
done
