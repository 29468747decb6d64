#!/bin/bash
# GPU parity tests, then a bench argument sweep. Usage: TAG=x ARGSETS="--a;--b" bash tools/gpu_test_sweep.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-ts}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
TAG=${TAG:-ts} bash tools/gpu_sweep.sh
