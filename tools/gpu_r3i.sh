#!/bin/bash
# GPU box: Quiver tests first, the full GPU suite, Quiver stage A/B (libbase.so vs the tree's library) and its
# kernel profile, the default bench, the configs[2] path trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3i}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_quiver_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_quiver.log 2>&1 || { echo "quiver pytest failed"; tail -40 $OUT/pytest_quiver.log; exit 1; }
tail -1 $OUT/pytest_quiver.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for i in 1 2; do
  for l in libbase libpbccs_amd; do
    PBCCS_LIB=$GRAFT_REPO_ROOT/pbccs_amd/_lib/$l.so timeout -k 10 300 python -u bench.py --stage quiver --steps 1 --warmup 1 --cpu-sample 0 > $OUT/q_${l}_$i.json 2> $OUT/q_${l}_$i.err || { echo "quiver $l failed"; tail -20 $OUT/q_${l}_$i.err; exit 1; }
    echo "quiver $l: $(python -c "import json; d=json.load(open('$OUT/q_${l}_$i.json')); print(d['value'], d['converged'], d['mean_iterations_applied'])")"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/qprof -o qprof -- python3 -u bench.py --stage quiver --steps 1 --warmup 1 --cpu-sample 0 > $OUT/quiver_prof.json 2> $OUT/quiver_prof.err || { echo "quiver prof failed"; tail -20 $OUT/quiver_prof.err; exit 1; }
for i in 1 2; do
  for l in libbase libpbccs_amd; do
    PBCCS_LIB=$GRAFT_REPO_ROOT/pbccs_amd/_lib/$l.so timeout -k 10 300 python -u bench.py --cpu-sample 0 > $OUT/p_${l}_$i.json 2> $OUT/p_${l}_$i.err || { echo "bench $l failed"; tail -20 $OUT/p_${l}_$i.err; exit 1; }
    echo "2kb $l: $(python -c "import json; d=json.load(open('$OUT/p_${l}_$i.json')); k=d['kernels']['k_score']; print(d['value'], d['zmw_status'], 'k_score', round(k['device_ms']/k['launches'],2), 'ms/launch')")"
  done
done
PBCCS_FILL_PATHS=1 PBCCS_ROUND_TRACE=1 timeout -k 10 600 python -u bench.py --workload 10kb --steps 4 --zmws-per-step 60 --warmup 0 --cpu-sample 0 > $OUT/trace10.json 2> $OUT/trace10.err || { echo "10kb trace failed"; tail -20 $OUT/trace10.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/trace10.json')); print('10kb', d['value'], d['zmw_status'])"
