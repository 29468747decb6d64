#!/bin/bash
# GPU box: POA tests, then an interleaved A/B of the POA stage and the ccs stage between the HEAD build
# (libbase.so) and the working tree (persistent host worker pool, reused column programs).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3u}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_poa_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_poa.log 2>&1 || { echo "poa pytest failed"; tail -40 $OUT/pytest_poa.log; exit 1; }
tail -1 $OUT/pytest_poa.log
BASE=$PWD/pbccs_amd/_lib/libbase.so
stage() {   # name stage lib
  local name=$1 st=$2 lib=$3
  PBCCS_LIB=$lib timeout -k 10 300 python -u bench.py --stage $st --steps 5 --warmup 1 --cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -20 $OUT/$name.err; return 1; }
  echo "$name: $(python -c "import json; d=json.load(open('$OUT/$name.json')); p=d.get('poa',{}).get('host_ms') or {k: d.get(k) for k in ('poa_wall_ms','poa_device_ms','poa_thread_ms')}; print(d['value'], d['ms_per_step'], p)")"
}
stage poa_new poa "" && stage poa_base poa $BASE && stage poa_new2 poa "" && stage poa_base2 poa $BASE && \
stage ccs_new ccs "" && stage ccs_base ccs $BASE
