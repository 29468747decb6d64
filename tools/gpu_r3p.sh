#!/bin/bash
# GPU box: POA tests (traceback with LDS-staged column programs) and the POA stage; the Quiver stage with its
# phase trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3p}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_poa_gpu.py tests/test_driver.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_poa.log 2>&1 || { echo "poa pytest failed"; tail -40 $OUT/pytest_poa.log; exit 1; }
tail -1 $OUT/pytest_poa.log
timeout -k 10 300 python -u bench.py --stage poa --steps 5 --warmup 1 --cpu-sample 0 > $OUT/poa.json 2> $OUT/poa.err || { echo "poa failed"; tail -20 $OUT/poa.err; exit 1; }
echo "poa: $(python -c "import json; d=json.load(open('$OUT/poa.json')); print(d['value'], d['poa'])")"
PBCCS_QUIVER_TRACE=1 timeout -k 10 300 python -u bench.py --stage quiver --steps 5 --warmup 1 --cpu-sample 0 > $OUT/quiver5.json 2> $OUT/quiver5.err || { echo "quiver failed"; tail -20 $OUT/quiver5.err; exit 1; }
echo "quiver 5 steps: $(python -c "import json; d=json.load(open('$OUT/quiver5.json')); print(d['value'], d['ms_per_step'])")"
grep '\[quiver\]' $OUT/quiver5.err | tail -20
