#!/bin/bash
# one-off: single-slot rocprof + PMC pass 1 for the main and the A/B library (k_score guard-free split)
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4m; mkdir -p $OUT
for v in main ab; do
  L=pbccs_amd/_lib/libpbccs_amd.so; [ $v = ab ] && L=pbccs_amd/_lib_ab/libpbccs_amd.so
  PBCCS_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof1_$v -o run -- python3 -u bench.py --streams 1 --steps 5 --warmup 1 --cpu-sample 0 > $OUT/s1_$v.json 2> $OUT/s1_$v.err || exit 1
  echo "$v $(python3 -c "import json; d=json.load(open('$OUT/s1_$v.json')); print(d['value'])")"
  PBCCS_LIB=$L timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU -f csv -d $OUT/pmc_$v -o pmc -- python3 -u bench.py --cpu-sample 0 --no-profile --steps 3 --warmup 1 > $OUT/pmc_$v.json 2> $OUT/pmc_$v.err || exit 1
  python3 tools/pmc_summary.py $(find $OUT/pmc_$v -name '*counter_collection.csv') > $OUT/pmc_$v.txt || exit 1
  grep -A8 "== k_score" $OUT/pmc_$v.txt | grep -E "==|INSTS_VALU|WAVE_CYCLES" 
done
