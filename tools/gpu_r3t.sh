#!/bin/bash
# GPU box: Quiver stage A/B over the coop fill's LDS ring height (PBCCS_QRING_ROWS) and feature window (libw128.so:
# kQWinRows 128), with the fill trace (tall re-runs) and the phase trace; engine-cached QuiverBatch.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3t}
mkdir -p $OUT
run() {   # name, env...
  local name=$1; shift
  env "$@" PBCCS_QUIVER_TRACE=1 PBCCS_QFILL_TRACE=1 timeout -k 10 240 python -u bench.py --stage quiver --steps 5 --warmup 1 --cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -20 $OUT/$name.err; return 1; }
  echo "$name: $(python -c "import json; d=json.load(open('$OUT/$name.json')); print(d['value'], d['ms_per_step'])") tall=$(grep -c 'tall [1-9]' $OUT/$name.err)"
}
timeout -k 10 300 python -u -m pytest tests/test_quiver_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_quiver.log 2>&1 || { echo "quiver pytest failed"; tail -40 $OUT/pytest_quiver.log; exit 1; }
tail -1 $OUT/pytest_quiver.log
run ring1024 PBCCS_QRING_ROWS=1024 && \
run ring256 PBCCS_QRING_ROWS=256 && \
run ring512 PBCCS_QRING_ROWS=512 && \
run w128_ring256 PBCCS_LIB=$PWD/pbccs_amd/_lib/libw128.so PBCCS_QRING_ROWS=256 && \
run w128_ring512 PBCCS_LIB=$PWD/pbccs_amd/_lib/libw128.so PBCCS_QRING_ROWS=512 && \
run w128_ring128 PBCCS_LIB=$PWD/pbccs_amd/_lib/libw128.so PBCCS_QRING_ROWS=128 && \
run w128_ring64 PBCCS_LIB=$PWD/pbccs_amd/_lib/libw128.so PBCCS_QRING_ROWS=64 && \
grep '\[quiver\]' $OUT/ring1024.err | tail -9
