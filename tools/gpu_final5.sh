#!/bin/bash
# GPU box, final evidence at the final sources: part 1 (GPU suite, smoke, driver bench, rocprof, traffic passes)
# then the Quiver / POA / ccs stage lines with CPU baselines and the Quiver kernel summary.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TAG=f5 bash tools/gpu_final1.sh || exit 1
OUT=gpurun_out/f5s
mkdir -p $OUT
PBCCS_QUIVER_TRACE=1 timeout -k 10 300 python -u bench.py --stage quiver --steps 5 --warmup 1 --cpu-sample 64 > $OUT/quiver.json 2> $OUT/quiver.err || { echo "quiver failed"; tail -20 $OUT/quiver.err; exit 1; }
echo "quiver: $(python -c "import json; d=json.load(open('$OUT/quiver.json')); print(d['value'], d['cpu_baseline']['value'])")"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/qprof -o qprof -- python3 -u bench.py --stage quiver --steps 5 --warmup 1 --cpu-sample 0 > $OUT/quiver_prof.json 2> $OUT/quiver_prof.err || { echo "quiver prof failed"; tail -20 $OUT/quiver_prof.err; exit 1; }
echo "quiver (rocprof): $(python -c "import json; d=json.load(open('$OUT/quiver_prof.json')); print(d['value'])")"
timeout -k 10 400 python -u bench.py --stage poa --steps 5 --warmup 1 > $OUT/poa.json 2> $OUT/poa.err || { echo "poa failed"; tail -20 $OUT/poa.err; exit 1; }
echo "poa: $(python -c "import json; d=json.load(open('$OUT/poa.json')); print(d['value'], d.get('cpu_baseline',{}).get('value'), d.get('vs_cpu'))")"
PBCCS_CCS_TRACE=1 timeout -k 10 500 python -u bench.py --stage ccs --steps 5 --warmup 1 > $OUT/ccs.json 2> $OUT/ccs.err || { echo "ccs failed"; tail -20 $OUT/ccs.err; exit 1; }
echo "ccs: $(python -c "import json; d=json.load(open('$OUT/ccs.json')); print(d['value'], d['zmw_status'], d.get('cpu_baseline',{}).get('value'), d.get('vs_cpu'))")"
