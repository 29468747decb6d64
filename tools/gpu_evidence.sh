#!/bin/bash
# Counter evidence at HEAD on the headline workload: two SQ/GRBM PMC groups (VALU busy, issue stalls, LDS
# bank conflicts per kernel) and the FETCH_SIZE / WRITE_SIZE traffic passes of the roofline kernel.
# Usage: TAG=x bash tools/gpu_evidence.sh   (BENCH_ARGS default: --steps 5 --warmup 1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export BENCH_ARGS="${BENCH_ARGS:---steps 5 --warmup 1}"
TAG=${TAG:-evidence}_pmc bash tools/gpu_pmc.sh || exit 1
python3 tools/pmc_summary.py gpurun_out/${TAG:-evidence}_pmc/pmc*/pmc*counter_collection.csv > gpurun_out/${TAG:-evidence}_pmc/summary.txt 2>&1 || true
find gpurun_out/${TAG:-evidence}_pmc -name "*counter_collection.csv" -exec gzip -f {} \;
TAG=${TAG:-evidence}_traffic bash tools/gpu_traffic.sh || exit 1
