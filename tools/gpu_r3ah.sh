#!/bin/bash
# GPU box: POA tests, then the POA stage three times (column-wise POA marshalling in pbccs_amd.poa).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3ah}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_poa_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_poa.log 2>&1 || { echo "poa pytest failed"; tail -40 $OUT/pytest_poa.log; exit 1; }
tail -1 $OUT/pytest_poa.log
for k in 1 2 3; do
  timeout -k 10 300 python -u bench.py --stage poa --steps 5 --warmup 1 --cpu-sample 0 > $OUT/poa$k.json 2> $OUT/poa$k.err || { echo "poa$k failed"; tail -20 $OUT/poa$k.err; exit 1; }
  echo "poa$k: $(python -c "import json; d=json.load(open('$OUT/poa$k.json')); print(d['value'], d['ms_per_step'], d['poa']['host_ms'])")"
done
