#!/bin/bash
# GPU box: Quiver tests with k_qfill_grp (four reads per wave) on by default, then the Quiver stage A/B:
# grouped fill on / off (PBCCS_QFILL_GRP=0), coop ring 128 / 256, with the fill trace (tall re-runs).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3x}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_quiver_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_quiver.log 2>&1 || { echo "quiver pytest failed"; tail -40 $OUT/pytest_quiver.log; exit 1; }
tail -1 $OUT/pytest_quiver.log
run() {   # name, env...
  local name=$1; shift
  env "$@" PBCCS_QUIVER_TRACE=1 PBCCS_QFILL_TRACE=1 timeout -k 10 240 python -u bench.py --stage quiver --steps 5 --warmup 1 --cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -20 $OUT/$name.err; return 1; }
  echo "$name: $(python -c "import json; d=json.load(open('$OUT/$name.json')); print(d['value'], d['ms_per_step'])")"
}
run grp_r128 PBCCS_QRING_ROWS=128 && run nogrp_r128 PBCCS_QFILL_GRP=0 PBCCS_QRING_ROWS=128 && \
run grp_r256 PBCCS_QRING_ROWS=256 && run nogrp_r128b PBCCS_QFILL_GRP=0 PBCCS_QRING_ROWS=128 && run grp_r128b PBCCS_QRING_ROWS=128 && \
grep '\[qfill\]' $OUT/grp_r128.err | tail -12 && grep '\[quiver\]' $OUT/grp_r128.err | tail -9
