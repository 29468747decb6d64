#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprof kernel summary. Each GPU step has its own limit.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-run}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o prof -- python3 -u bench.py --cpu-sample 0 ${BENCH_ARGS} > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { echo rocprof failed; tail -30 $OUT/prof_bench.err; exit 1; }
find $OUT/prof -name "*stats*"
