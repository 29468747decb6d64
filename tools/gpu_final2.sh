#!/bin/bash
# GPU box, final evidence part 2 (sources frozen): single-slot kernel summary, SQ PMC groups, the Quiver, POA and
# ccs stage lines (CPU baselines in each) and the Quiver kernel summary.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-f2}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof1 -o prof -- python3 -u bench.py --gpus 1 --steps 5 --warmup 1 --streams 1 --cpu-sample 0 > $OUT/bench_streams1.json 2> $OUT/bench_streams1.err || { echo "streams1 failed"; tail -20 $OUT/bench_streams1.err; exit 1; }
echo "streams1: $(python -c "import json; d=json.load(open('$OUT/bench_streams1.json')); print(d['value'], d['ms_per_step'])")"
TAG=${TAG:-f2}_pmc bash tools/gpu_pmc.sh || exit 1
python3 tools/pmc_summary.py gpurun_out/${TAG:-f2}_pmc/pmc*/pmc*counter_collection.csv > gpurun_out/${TAG:-f2}_pmc/summary.txt 2>&1 || true
find gpurun_out/${TAG:-f2}_pmc -name "*counter_collection.csv" -exec gzip -f {} \;
timeout -k 10 300 python -u bench.py --stage quiver --steps 5 --warmup 1 --cpu-sample 64 > $OUT/quiver.json 2> $OUT/quiver.err || { echo "quiver failed"; tail -20 $OUT/quiver.err; exit 1; }
echo "quiver: $(python -c "import json; d=json.load(open('$OUT/quiver.json')); print(d['value'], d['cpu_baseline']['value'])")"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/qprof -o qprof -- python3 -u bench.py --stage quiver --steps 5 --warmup 1 --cpu-sample 0 > $OUT/quiver_prof.json 2> $OUT/quiver_prof.err || { echo "quiver prof failed"; tail -20 $OUT/quiver_prof.err; exit 1; }
timeout -k 10 400 python -u bench.py --stage poa --steps 5 --warmup 1 > $OUT/poa.json 2> $OUT/poa.err || { echo "poa failed"; tail -20 $OUT/poa.err; exit 1; }
echo "poa: $(python -c "import json; d=json.load(open('$OUT/poa.json')); print(d['value'], d.get('cpu_baseline',{}).get('value'), d.get('vs_cpu'))")"
PBCCS_CCS_TRACE=1 timeout -k 10 500 python -u bench.py --stage ccs --steps 5 --warmup 1 > $OUT/ccs.json 2> $OUT/ccs.err || { echo "ccs failed"; tail -20 $OUT/ccs.err; exit 1; }
echo "ccs: $(python -c "import json; d=json.load(open('$OUT/ccs.json')); print(d['value'], d['zmw_status'], d.get('cpu_baseline',{}).get('value'), d.get('vs_cpu'))")"
