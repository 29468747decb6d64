#!/bin/bash
# rocprofv3 kernel summaries of a short bench for each variant (env settings separated by ';').
# Usage: TAG=x VARIANTS="A=1;B=2" BENCH_ARGS="--steps 2" bash tools/gpu_prof_ab.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-profab}
mkdir -p $OUT
i=0
IFS=';' read -ra VS <<< "${VARIANTS:-X=0}"
for v in "${VS[@]}"; do
  i=$((i+1))
  echo "== variant $i: $v"
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/p$i -o prof -- python3 -u bench.py --cpu-sample 0 ${BENCH_ARGS} > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { echo "variant $i failed"; tail -20 $OUT/bench_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$i.json')); print(d['value'], d['kernels']['k_fill'], d['kernels']['k_score'])"
  f=$(find $OUT/p$i -name "*kernel_stats.csv" | head -1)
  cut -d, -f1-4 "$f" | head -8
  find $OUT/p$i -name "*kernel_trace.csv" -exec gzip -f {} \;
done
