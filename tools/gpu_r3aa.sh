#!/bin/bash
# GPU box: ccs stage A/B over the polish units (PBCCS_CCS_SPLIT pieces per chunk, PBCCS_CCS_TAIL_SPLIT for the
# last chunk), with the chunk trace; the POA GPU tests first (pbccs_ccs_batch parity).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3aa}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_poa_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_poa.log 2>&1 || { echo "poa pytest failed"; tail -40 $OUT/pytest_poa.log; exit 1; }
tail -1 $OUT/pytest_poa.log
run() {   # name, env...
  local name=$1; shift
  env "$@" PBCCS_CCS_TRACE=1 timeout -k 10 300 python -u bench.py --stage ccs --steps 5 --warmup 1 --cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -20 $OUT/$name.err; return 1; }
  echo "$name: $(python -c "import json; d=json.load(open('$OUT/$name.json')); print(d['value'], d['ms_per_step'], d['zmw_status'])")"
}
run s1t1 PBCCS_CCS_SPLIT=1 PBCCS_CCS_TAIL_SPLIT=1 && run s1t5 PBCCS_CCS_SPLIT=1 PBCCS_CCS_TAIL_SPLIT=5 && \
run s2t4 PBCCS_CCS_SPLIT=2 PBCCS_CCS_TAIL_SPLIT=4 && run s2t2 PBCCS_CCS_SPLIT=2 PBCCS_CCS_TAIL_SPLIT=2 && \
run s1t1b PBCCS_CCS_SPLIT=1 PBCCS_CCS_TAIL_SPLIT=1 && run s1t5b PBCCS_CCS_SPLIT=1 PBCCS_CCS_TAIL_SPLIT=5 && \
grep '\[ccs\]' $OUT/s1t5.err | tail -14
