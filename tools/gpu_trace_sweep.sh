#!/bin/bash
# GPU parity tests, then bench runs with the per-round trace, one per ';'-separated "ENV... -- ARGS" variant.
# Usage: TAG=x VARIANTS="PBCCS_X=0 -- --steps 10;-- --streams 7" bash tools/gpu_trace_sweep.sh  (SKIP_TESTS=1 skips pytest)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-trace}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
i=0
IFS=';' read -ra VS <<< "${VARIANTS:-}"
for v in "${VS[@]}"; do
  i=$((i+1))
  envs="${v%%--*}"
  args="${v#*--}"
  echo "== variant $i: env [$envs] args [$args]"
  env PBCCS_ROUND_TRACE=1 $envs timeout -k 10 300 python -u bench.py --cpu-sample 0 --no-profile $args > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { echo bench failed; tail -20 $OUT/bench_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$i.json')); print(d['value'], d['ms_per_step'], d['zmw_status'], d['band_memory_gb'], d.get('oom_retries'))"
done
