#!/bin/bash
# A/B bench runs on the GPU box (no profiler). Usage: TAG=x VARIANTS="env1;env2" bash tools/gpu_bench_ab.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
i=0
IFS=';' read -ra VS <<< "${VARIANTS:-}"
for v in "${VS[@]}"; do
  i=$((i+1))
  echo "== variant $i: $v"
  env $v timeout -k 10 300 python -u bench.py --cpu-sample 0 ${BENCH_ARGS} > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { echo bench failed; tail -20 $OUT/bench_$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_$i.json')); print(d['value'], d['ms_per_step'], d['zmw_status'], d['roofline']['avg_launch_ms'])"
done
