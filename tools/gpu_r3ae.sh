#!/bin/bash
# GPU box: Quiver tests; Quiver stage A/B (grp-tall reads' arenas pre-sized vs HEAD libbase.so); the traffic
# passes at the working tree's sources.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3ae}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_quiver_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_quiver.log 2>&1 || { echo "quiver pytest failed"; tail -40 $OUT/pytest_quiver.log; exit 1; }
tail -1 $OUT/pytest_quiver.log
run() {   # name, env...
  local name=$1; shift
  env "$@" PBCCS_QUIVER_TRACE=1 PBCCS_QFILL_TRACE=1 timeout -k 10 240 python -u bench.py --stage quiver --steps 5 --warmup 1 --cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -20 $OUT/$name.err; return 1; }
  echo "$name: $(python -c "import json; d=json.load(open('$OUT/$name.json')); print(d['value'], d['ms_per_step'])")"
}
BASE=$PWD/pbccs_amd/_lib/libbase.so
run presize && run base PBCCS_LIB=$BASE && run presize2 && run base2 PBCCS_LIB=$BASE && \
grep '\[qfill\]\|addreads\|round [0-2] ' $OUT/presize2.err | tail -12 && \
BENCH_ARGS="--steps 5 --warmup 1" TAG=r3ae_traffic bash tools/gpu_traffic.sh > /dev/null && echo "traffic ok"
