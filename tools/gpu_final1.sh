#!/bin/bash
# GPU box, final evidence part 1 (sources frozen): the full GPU suite, smoke(), the driver's bench command, its
# rocprofv3 kernel summary, and the FETCH_SIZE / WRITE_SIZE traffic passes of the roofline kernels.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-f1}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
echo "bench: $(python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['gcups'], d['cpu_baseline']['value'])")"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o prof -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "bench prof failed"; tail -20 $OUT/bench_prof.err; exit 1; }
echo "bench (rocprof): $(python -c "import json; d=json.load(open('$OUT/bench_prof.json')); print(d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'])")"
BENCH_ARGS="--steps 5 --warmup 1" TAG=${TAG:-f1}_traffic bash tools/gpu_traffic.sh || exit 1
