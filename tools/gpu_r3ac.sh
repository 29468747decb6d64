#!/bin/bash
# GPU box: Quiver tests; Quiver stage A/B (grp-tall reads straight to the full-height ring vs HEAD libbase.so);
# the ccs chunk-size A/B (tools/gpu_r3ab.sh); the traffic passes at the working tree's sources.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3ac}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_quiver_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_quiver.log 2>&1 || { echo "quiver pytest failed"; tail -40 $OUT/pytest_quiver.log; exit 1; }
tail -1 $OUT/pytest_quiver.log
run() {   # name, env...
  local name=$1; shift
  env "$@" PBCCS_QUIVER_TRACE=1 PBCCS_QFILL_TRACE=1 timeout -k 10 240 python -u bench.py --stage quiver --steps 5 --warmup 1 --cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -20 $OUT/$name.err; return 1; }
  echo "$name: $(python -c "import json; d=json.load(open('$OUT/$name.json')); print(d['value'], d['ms_per_step'])")"
}
BASE=$PWD/pbccs_amd/_lib/libbase.so
run full && run base PBCCS_LIB=$BASE && run full2 && run base2 PBCCS_LIB=$BASE && \
TAG=r3ab bash tools/gpu_r3ab.sh && \
BENCH_ARGS="--steps 5 --warmup 1" TAG=r3ac_traffic bash tools/gpu_traffic.sh > /dev/null && echo "traffic ok"
