#!/bin/bash
# GPU box: checkpointed-band parity (tests/test_ckpt_gpu.py + the 10 kb / 15 kb fixture tests), then the
# configs[2] queue bench with checkpoints off and on.  Usage: TAG=x N=480 bash tools/gpu_ckpt.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-ckpt}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_ckpt_gpu.py tests/test_gpu_parity.py -k "ckpt or checkpoint or 10kb or mixed_long" -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
[ -n "$SKIP_BENCH" ] && exit 0
N=${N:-480}
for k in ${CKPT_KS:-0 8}; do
  PBCCS_CKPT_K=$k timeout -k 10 600 python -u bench.py --workload 10kb --steps 8 --zmws-per-step $((N / 8)) --warmup 0 --cpu-sample 0 > $OUT/bench10_k$k.json 2> $OUT/bench10_k$k.err || { echo "bench K=$k failed"; tail -20 $OUT/bench10_k$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench10_k$k.json')); print('K=$k', d['value'], d['gcups'], d['zmw_status'], d['band_memory_gb'], d['config']['slots'])"
done
