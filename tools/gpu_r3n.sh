#!/bin/bash
# GPU box: full GPU suite; Quiver stage (5 steps); configs[2] at 2000 ZMWs with the round trace; the POA and
# end-to-end ccs stage lines with their CPU baselines.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3n}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
PBCCS_QFILL_TRACE=1 timeout -k 10 300 python -u bench.py --stage quiver --steps 5 --warmup 1 --cpu-sample 0 > $OUT/quiver5.json 2> $OUT/quiver5.err || { echo "quiver failed"; tail -20 $OUT/quiver5.err; exit 1; }
echo "quiver 5 steps: $(python -c "import json; d=json.load(open('$OUT/quiver5.json')); print(d['value'], d['ms_per_step'])")"
PBCCS_ROUND_TRACE=1 PBCCS_FILL_PATHS=1 timeout -k 10 700 python -u bench.py --workload 10kb --steps 8 --zmws-per-step 250 --warmup 0 --cpu-sample 0 > $OUT/bench_10kb_2000.json 2> $OUT/bench_10kb_2000.err || { echo "10kb failed"; tail -20 $OUT/bench_10kb_2000.err; exit 1; }
echo "10kb x2000: $(python -c "import json; d=json.load(open('$OUT/bench_10kb_2000.json')); print(d['value'], d['gcups'], d['zmw_status'], d['band_memory_gb']['pool_mapped_bytes'])")"
timeout -k 10 400 python -u bench.py --stage poa --steps 5 --warmup 1 > $OUT/poa.json 2> $OUT/poa.err || { echo "poa failed"; tail -20 $OUT/poa.err; exit 1; }
echo "poa: $(python -c "import json; d=json.load(open('$OUT/poa.json')); print(d['value'], d.get('cpu_baseline',{}).get('value'), d.get('vs_cpu'))")"
timeout -k 10 500 python -u bench.py --stage ccs --steps 5 --warmup 1 > $OUT/ccs.json 2> $OUT/ccs.err || { echo "ccs failed"; tail -20 $OUT/ccs.err; exit 1; }
echo "ccs: $(python -c "import json; d=json.load(open('$OUT/ccs.json')); print(d['value'], d['zmw_status'], d.get('cpu_baseline',{}).get('value'), d.get('vs_cpu'))")"
