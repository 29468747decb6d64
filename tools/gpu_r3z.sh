#!/bin/bash
# GPU box: Quiver tests; Quiver stage A/B (tall fills on a side stream vs HEAD's libbase.so); then the ccs
# POA-slice A/B (tools/gpu_r3y.sh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3z}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_quiver_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_quiver.log 2>&1 || { echo "quiver pytest failed"; tail -40 $OUT/pytest_quiver.log; exit 1; }
tail -1 $OUT/pytest_quiver.log
run() {   # name, env...
  local name=$1; shift
  env "$@" PBCCS_QUIVER_TRACE=1 timeout -k 10 240 python -u bench.py --stage quiver --steps 5 --warmup 1 --cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -20 $OUT/$name.err; return 1; }
  echo "$name: $(python -c "import json; d=json.load(open('$OUT/$name.json')); print(d['value'], d['ms_per_step'])")"
}
BASE=$PWD/pbccs_amd/_lib/libbase.so
run side && run base PBCCS_LIB=$BASE && run side2 && run base2 PBCCS_LIB=$BASE && \
grep '\[quiver\]' $OUT/side2.err | grep -v deltas | tail -8 && TAG=r3y bash tools/gpu_r3y.sh
