#!/bin/bash
# GPU box: Quiver tests, the Quiver stage (5 steps, trace) and its kernel profile.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3s}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_quiver_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_quiver.log 2>&1 || { echo "quiver pytest failed"; tail -40 $OUT/pytest_quiver.log; exit 1; }
tail -1 $OUT/pytest_quiver.log
PBCCS_QUIVER_TRACE=1 timeout -k 10 300 python -u bench.py --stage quiver --steps 5 --warmup 1 --cpu-sample 0 > $OUT/quiver5.json 2> $OUT/quiver5.err || { echo "quiver failed"; tail -20 $OUT/quiver5.err; exit 1; }
echo "quiver 5 steps: $(python -c "import json; d=json.load(open('$OUT/quiver5.json')); print(d['value'], d['ms_per_step'])")"
grep '\[quiver\]' $OUT/quiver5.err | tail -9
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/qprof -o qprof -- python3 -u bench.py --stage quiver --steps 5 --warmup 1 --cpu-sample 64 > $OUT/quiver_prof.json 2> $OUT/quiver_prof.err || { echo "quiver prof failed"; tail -20 $OUT/quiver_prof.err; exit 1; }
echo "quiver (rocprof, cpu baseline): $(python -c "import json; d=json.load(open('$OUT/quiver_prof.json')); print(d['value'], d.get('cpu_baseline'))")"
