#!/bin/bash
# Work-queue pass on the GPU box: scheduler parity, a short default bench, configs[3] mixed and configs[2]
# 10 kb through polish_stream.  Each GPU step has its own limit.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-queue}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_schedule.py -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_queue.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_queue.log; exit 1; }
tail -2 $OUT/pytest_queue.log
timeout -k 10 200 python -u bench.py --steps 2 --zmws-per-step 500 --cpu-sample 0 > $OUT/bench_short.json 2> $OUT/bench_short.err || { echo short bench failed; tail -20 $OUT/bench_short.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_short.json')); print('2kb', d['value'])"
timeout -k 10 ${MIXED_LIMIT:-420} python -u bench.py --workload mixed --steps 1 --zmws-per-step ${MIXED_N:-100} --streams 4 > $OUT/bench_mixed.json 2> $OUT/bench_mixed.err || { echo mixed bench failed; tail -20 $OUT/bench_mixed.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_mixed.json')); print('mixed', d['value'], d['zmw_status'])"
timeout -k 10 ${TENKB_LIMIT:-300} python -u bench.py --workload 10kb --steps 1 --zmws-per-step ${TENKB_N:-120} --streams 4 > $OUT/bench_10kb.json 2> $OUT/bench_10kb.err || { echo 10kb bench failed; tail -20 $OUT/bench_10kb.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_10kb.json')); print('10kb', d['value'], d['zmw_status'])"
