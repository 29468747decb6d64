#!/bin/bash
# GPU box, final check at the frozen sources (traffic profiles already match them): GPU suite, smoke, driver bench,
# its rocprof summary, the Quiver / POA / ccs stage lines, then the configs[2] slot A/B (tools/gpu_r3ad.sh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/f4
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
echo "bench: $(python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['gcups'], d['cpu_baseline']['value'], d['roofline']['traffic'], d['roofline']['traffic_source'])")"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o prof -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "bench prof failed"; tail -20 $OUT/bench_prof.err; exit 1; }
echo "bench (rocprof): $(python -c "import json; d=json.load(open('$OUT/bench_prof.json')); print(d['value'])")"
PBCCS_QUIVER_TRACE=1 timeout -k 10 300 python -u bench.py --stage quiver --steps 5 --warmup 1 --cpu-sample 64 > $OUT/quiver.json 2> $OUT/quiver.err || { echo "quiver failed"; tail -20 $OUT/quiver.err; exit 1; }
echo "quiver: $(python -c "import json; d=json.load(open('$OUT/quiver.json')); print(d['value'], d['cpu_baseline']['value'])")"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/qprof -o qprof -- python3 -u bench.py --stage quiver --steps 5 --warmup 1 --cpu-sample 0 > $OUT/quiver_prof.json 2> $OUT/quiver_prof.err || { echo "quiver prof failed"; tail -20 $OUT/quiver_prof.err; exit 1; }
timeout -k 10 400 python -u bench.py --stage poa --steps 5 --warmup 1 > $OUT/poa.json 2> $OUT/poa.err || { echo "poa failed"; tail -20 $OUT/poa.err; exit 1; }
echo "poa: $(python -c "import json; d=json.load(open('$OUT/poa.json')); print(d['value'], d.get('cpu_baseline',{}).get('value'), d.get('vs_cpu'))")"
PBCCS_CCS_TRACE=1 timeout -k 10 500 python -u bench.py --stage ccs --steps 5 --warmup 1 > $OUT/ccs.json 2> $OUT/ccs.err || { echo "ccs failed"; tail -20 $OUT/ccs.err; exit 1; }
echo "ccs: $(python -c "import json; d=json.load(open('$OUT/ccs.json')); print(d['value'], d['zmw_status'], d.get('cpu_baseline',{}).get('value'), d.get('vs_cpu'))")"
TAG=r3ad bash tools/gpu_r3ad.sh
