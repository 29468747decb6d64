#!/bin/bash
# GPU box: Quiver tests, Quiver stage A/B (libbase.so vs the tree's library) + kernel profile; then configs[2] at
# 2000 ZMWs, a single-slot rocprofv3 kernel summary of the 2 kb bench, the configs[4] two-rank rehearsal.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3k}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_quiver_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_quiver.log 2>&1 || { echo "quiver pytest failed"; tail -40 $OUT/pytest_quiver.log; exit 1; }
tail -1 $OUT/pytest_quiver.log
for i in 1 2; do
  for l in libbase libpbccs_amd; do
    PBCCS_LIB=$GRAFT_REPO_ROOT/pbccs_amd/_lib/$l.so timeout -k 10 300 python -u bench.py --stage quiver --steps 1 --warmup 1 --cpu-sample 0 > $OUT/q_${l}_$i.json 2> $OUT/q_${l}_$i.err || { echo "quiver $l failed"; tail -20 $OUT/q_${l}_$i.err; exit 1; }
    echo "quiver $l: $(python -c "import json; d=json.load(open('$OUT/q_${l}_$i.json')); print(d['value'], d['converged'], d['mean_iterations_applied'])")"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/qprof -o qprof -- python3 -u bench.py --stage quiver --steps 1 --warmup 1 --cpu-sample 0 > $OUT/quiver_prof.json 2> $OUT/quiver_prof.err || { echo "quiver prof failed"; tail -20 $OUT/quiver_prof.err; exit 1; }
TAG=${TAG:-r3k} bash tools/gpu_r3j.sh
