#!/bin/bash
# GPU box: ccs stage A/B over the POA slice count (PBCCS_POA_SLICES) with the chunk trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3y}
mkdir -p $OUT
run() {   # name, env...
  local name=$1; shift
  env "$@" PBCCS_CCS_TRACE=1 timeout -k 10 300 python -u bench.py --stage ccs --steps 5 --warmup 1 --cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -20 $OUT/$name.err; return 1; }
  echo "$name: $(python -c "import json; d=json.load(open('$OUT/$name.json')); print(d['value'], d['ms_per_step'], d['poa_wall_ms'], d['poa_device_ms'], d['poa_thread_ms'])")"
}
run s2 PBCCS_POA_SLICES=2 && run s3 PBCCS_POA_SLICES=3 && run s4 PBCCS_POA_SLICES=4 && run s2b PBCCS_POA_SLICES=2 && run s1 PBCCS_POA_SLICES=1 && \
grep '\[ccs\]' $OUT/s2.err | tail -20
