#!/bin/bash
# GPU box: Quiver tests on the new defaults (ring 256, window 128, single-chunk register path), then the
# Quiver stage A/B against the window-128 build without the register path (libw128.so) and ring 128.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3v}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_quiver_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_quiver.log 2>&1 || { echo "quiver pytest failed"; tail -40 $OUT/pytest_quiver.log; exit 1; }
tail -1 $OUT/pytest_quiver.log
run() {   # name, env...
  local name=$1; shift
  env "$@" PBCCS_QUIVER_TRACE=1 timeout -k 10 240 python -u bench.py --stage quiver --steps 5 --warmup 1 --cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -20 $OUT/$name.err; return 1; }
  echo "$name: $(python -c "import json; d=json.load(open('$OUT/$name.json')); print(d['value'], d['ms_per_step'])")"
}
run new PBCCS_QRING_ROWS=256 && \
run w128_noreg PBCCS_LIB=$PWD/pbccs_amd/_lib/libw128.so PBCCS_QRING_ROWS=256 && \
run new_ring128 PBCCS_QRING_ROWS=128 && \
run new2 PBCCS_QRING_ROWS=256 && \
run w128_noreg2 PBCCS_LIB=$PWD/pbccs_amd/_lib/libw128.so PBCCS_QRING_ROWS=256 && \
grep '\[quiver\]' $OUT/new.err | tail -9
