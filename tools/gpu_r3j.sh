#!/bin/bash
# GPU box: configs[2] at 2000 ZMWs through the work queue; a single-slot rocprofv3 kernel summary of the 2 kb
# bench (kernel time per step <= ms_per_step); the configs[4] two-rank rehearsal on one device.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3j}
mkdir -p $OUT
PBCCS_FILL_PATHS=1 timeout -k 10 700 python -u bench.py --workload 10kb --steps 8 --zmws-per-step 250 --warmup 0 --cpu-sample 0 > $OUT/bench_10kb_2000.json 2> $OUT/bench_10kb_2000.err || { echo "10kb 2000 failed"; tail -20 $OUT/bench_10kb_2000.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_10kb_2000.json')); print('10kb x2000', d['value'], d['gcups'], d['zmw_status'], d['band_memory_gb'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof1 -o prof1 -- python3 -u bench.py --streams 1 --steps 4 --warmup 1 --cpu-sample 0 > $OUT/bench_streams1.json 2> $OUT/bench_streams1.err || { echo "streams1 prof failed"; tail -20 $OUT/bench_streams1.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_streams1.json')); print('streams1', d['value'], d['ms_per_step'])"
PBCCS_BENCH_DEVICE=0 timeout -k 10 600 python -u bench.py --gpus 2 --workload smrtcell --steps 4 --zmws-per-step 60 --streams 2 --warmup 0 --cpu-sample 0 > $OUT/bench_smrtcell_gpus2.json 2> $OUT/bench_smrtcell_gpus2.err || { echo "smrtcell failed"; tail -20 $OUT/bench_smrtcell_gpus2.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_smrtcell_gpus2.json')); print('smrtcell x2', d['value'], d['n_gpus'], d.get('queue'))"
