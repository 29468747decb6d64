#!/bin/bash
# GPU box: full GPU suite, the configs[2] path/round trace, the default bench, then a Quiver stage kernel profile.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3h}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
PBCCS_FILL_PATHS=1 PBCCS_ROUND_TRACE=1 timeout -k 10 600 python -u bench.py --workload 10kb --steps 4 --zmws-per-step 60 --warmup 0 --cpu-sample 0 > $OUT/trace10.json 2> $OUT/trace10.err || { echo "10kb trace failed"; tail -20 $OUT/trace10.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/trace10.json')); print('10kb', d['value'], d['zmw_status'])"
timeout -k 10 400 python -u bench.py --cpu-sample 0 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('2kb', d['value'], d['zmw_status'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/qprof -o qprof -- python3 -u bench.py --stage quiver --steps 1 --warmup 1 --cpu-sample 0 > $OUT/quiver.json 2> $OUT/quiver.err || { echo "quiver prof failed"; tail -20 $OUT/quiver.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/quiver.json')); print('quiver', d['value'])"
