#!/bin/bash
# GPU box: Quiver tests and stage (Jacobi cascade, ring sizes), Quiver kernel profile; configs[2] x1000 kernel
# profile (k_score / k_score_ckpt / fills split).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3o}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_quiver_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_quiver.log 2>&1 || { echo "quiver pytest failed"; tail -40 $OUT/pytest_quiver.log; exit 1; }
tail -1 $OUT/pytest_quiver.log
for rr in 1024 256; do
  PBCCS_QRING_ROWS=$rr timeout -k 10 300 python -u bench.py --stage quiver --steps 5 --warmup 1 --cpu-sample 0 > $OUT/q5_ring$rr.json 2> $OUT/q5_ring$rr.err || { echo "quiver ring $rr failed"; tail -20 $OUT/q5_ring$rr.err; exit 1; }
  echo "quiver 5 steps ring $rr: $(python -c "import json; d=json.load(open('$OUT/q5_ring$rr.json')); print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/qprof -o qprof -- python3 -u bench.py --stage quiver --steps 5 --warmup 1 --cpu-sample 0 > $OUT/quiver_prof.json 2> $OUT/quiver_prof.err || { echo "quiver prof failed"; tail -20 $OUT/quiver_prof.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof10 -o prof10 -- python3 -u bench.py --workload 10kb --steps 8 --zmws-per-step 125 --warmup 0 --cpu-sample 0 > $OUT/b10_prof.json 2> $OUT/b10_prof.err || { echo "10kb prof failed"; tail -20 $OUT/b10_prof.err; exit 1; }
echo "10kb x1000 (rocprof): $(python -c "import json; d=json.load(open('$OUT/b10_prof.json')); print(d['value'], d['gcups'])")"
