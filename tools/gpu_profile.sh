#!/bin/bash
# Bench with the per-round trace + a rocprofv3 kernel trace of the same command (GPU box).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-prof}
mkdir -p $OUT
PBCCS_ROUND_TRACE=1 timeout -k 10 300 python -u bench.py --cpu-sample 0 ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench_trace.err || { echo bench failed; tail -20 $OUT/bench_trace.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['zmw_status'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o prof -- python3 -u bench.py --cpu-sample 0 ${BENCH_ARGS} > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { echo rocprof failed; tail -20 $OUT/prof_bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/prof_bench.json')); print(d['value'], d['ms_per_step'])"
