#!/bin/bash
# GPU box: near-tall routing A/B (configs[2] x1000 and 2 kb), the lane-fill re-A/B under the current wave
# sorting, and the 12-slot mixed-240 command of round 1's std::terminate.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3m}
mkdir -p $OUT
for nt in 0 48; do
  PBCCS_NEAR_TALL=$nt PBCCS_FILL_PATHS=1 timeout -k 10 400 python -u bench.py --workload 10kb --steps 8 --zmws-per-step 125 --warmup 0 --cpu-sample 0 > $OUT/b10_nt$nt.json 2> $OUT/b10_nt$nt.err || { echo "10kb nt $nt failed"; tail -20 $OUT/b10_nt$nt.err; exit 1; }
  echo "10kb x1000 near-tall $nt: $(python -c "import json; d=json.load(open('$OUT/b10_nt$nt.json')); print(d['value'], d['gcups'], d['zmw_status'], d['band_memory_gb']['pool_mapped_bytes'])") attempt1-launches $(grep -c 'attempt=1' $OUT/b10_nt$nt.err)"
done
for i in 1 2; do
  for v in "PBCCS_NEAR_TALL=0" "PBCCS_NEAR_TALL=48" "PBCCS_FILL_LANE=1"; do
    env $v timeout -k 10 300 python -u bench.py --cpu-sample 0 --no-profile > $OUT/p_${v}_$i.json 2> $OUT/p_${v}_$i.err || { echo "bench $v failed"; tail -20 $OUT/p_${v}_$i.err; exit 1; }
    echo "2kb $v: $(python -c "import json; d=json.load(open('$OUT/p_${v}_$i.json')); print(d['value'], d['zmw_status'])")"
  done
done
timeout -k 10 900 python -u bench.py --workload mixed --steps 4 --zmws-per-step 60 --streams 12 --warmup 0 --cpu-sample 0 > $OUT/mixed240_s12.json 2> $OUT/mixed240_s12.err || { echo "mixed240 s12 failed rc=$?"; tail -20 $OUT/mixed240_s12.err; exit 1; }
echo "mixed240 s12: $(python -c "import json; d=json.load(open('$OUT/mixed240_s12.json')); print(d['value'], d['gcups'], d['zmw_status'], d['oom_retries'])")"
PBCCS_QRING_ROWS=1024 TAG=${TAG:-r3m}/qpmc BENCH_ARGS="--stage quiver --steps 1 --zmws-per-step 500 --warmup 0" bash tools/gpu_pmc.sh || exit 1
python3 tools/pmc_summary.py $(find gpurun_out/${TAG:-r3m}/qpmc -name '*counter_collection.csv') > gpurun_out/${TAG:-r3m}/qpmc_summary.txt && head -30 gpurun_out/${TAG:-r3m}/qpmc_summary.txt
