#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over a short bench. Usage: TAG=x bash tools/gpu_pmc.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-pmc}
mkdir -p $OUT
ARGS="--cpu-sample 0 --no-profile ${BENCH_ARGS:---steps 2 --zmws-per-step 500 --warmup 0}"
i=0
IFS=';' read -ra GROUPS_ <<< "${PMC_GROUPS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT}"
for g in "${GROUPS_[@]}"; do
  i=$((i+1))
  echo "== pass $i: $g"
  timeout -s KILL 240 rocprofv3 --pmc $g -f csv -d $OUT/pmc$i -o pmc -- python3 -u bench.py $ARGS > $OUT/pmc$i.json 2> $OUT/pmc$i.err || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.err; exit 1; }
done
