#!/bin/bash
# GPU box: ccs stage A/B over the chunk size (bench.py --ccs-chunk: ZMWs per POA chunk / polish batch), trace on.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3ab}
mkdir -p $OUT
run() {   # name, chunk
  local name=$1 chunk=$2
  PBCCS_CCS_TRACE=1 timeout -k 10 300 python -u bench.py --stage ccs --steps 5 --warmup 1 --cpu-sample 0 --ccs-chunk $chunk > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -20 $OUT/$name.err; return 1; }
  echo "$name: $(python -c "import json; d=json.load(open('$OUT/$name.json')); print(d['value'], d['ms_per_step'], d['zmw_status'])")"
}
run c2000 2000 && run c3334 3334 && run c5000 5000 && run c2500 2500 && run c2000b 2000 && run c3334b 3334 && \
grep '\[ccs\]' $OUT/c3334.err | tail -8
