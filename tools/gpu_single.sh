#!/bin/bash
# One batch, one stream: kernel trace + PMC passes to see per-launch latency and occupancy. TAG=x bash tools/gpu_single.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-single}
mkdir -p $OUT
ARGS="--cpu-sample 0 ${BENCH_ARGS:---steps 1 --warmup 0 --streams 1 --zmws-per-step 2000}"
PBCCS_ROUND_TRACE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/kt -o kt -- python3 -u bench.py $ARGS > $OUT/kt.json 2> $OUT/kt.err || { echo kt failed; tail -5 $OUT/kt.err; exit 1; }
grep '\[round\]' $OUT/kt.err
i=0
IFS=';' read -ra GROUPS_ <<< "${PMC_GROUPS:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_LDS;GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY}"
for g in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $g -f csv -d $OUT/pmc$i -o pmc -- python3 -u bench.py $ARGS --no-profile > $OUT/pmc$i.json 2> $OUT/pmc$i.err || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.err; exit 1; }
done
echo done
