#!/bin/bash
# GPU box: full GPU test suite, then interleaved A/B bench runs of an env switch.
# Usage: TAG=x AB_ENV="PBCCS_FOO=1" bash tools/gpu_ab.sh   (runs: A, B, A, B with B = AB_ENV set)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --cpu-sample 0 --no-profile > $OUT/a_$i.json 2> $OUT/a_$i.err || { echo bench A failed; tail -20 $OUT/a_$i.err; exit 1; }
  echo "A: $(python -c "import json; d=json.load(open('$OUT/a_$i.json')); print(d['value'], d['zmw_status'])")"
  env $AB_ENV timeout -k 10 300 python -u bench.py --cpu-sample 0 --no-profile > $OUT/b_$i.json 2> $OUT/b_$i.err || { echo bench B failed; tail -20 $OUT/b_$i.err; exit 1; }
  echo "B ($AB_ENV): $(python -c "import json; d=json.load(open('$OUT/b_$i.json')); print(d['value'], d['zmw_status'])")"
done
