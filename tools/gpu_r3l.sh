#!/bin/bash
# GPU box: full GPU suite; 2 kb A/B (libbase.so vs the tree's library); ccs stage with 2 vs 4 POA slices;
# configs[2] hybrid-path LDS rows A/B (3200 = the old budget vs the default cap).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3l}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for rr in 256 512 1024; do
  PBCCS_QFILL_TRACE=1 PBCCS_QRING_ROWS=$rr timeout -k 10 300 python -u bench.py --stage quiver --steps 1 --warmup 1 --cpu-sample 0 > $OUT/q_ring$rr.json 2> $OUT/q_ring$rr.err || { echo "quiver ring $rr failed"; tail -20 $OUT/q_ring$rr.err; exit 1; }
  echo "quiver ring $rr: $(python -c "import json; d=json.load(open('$OUT/q_ring$rr.json')); print(d['value'])") $(grep -c 'tall [1-9]' $OUT/q_ring$rr.err) launches with tall reads; $(grep qfill $OUT/q_ring$rr.err | head -3 | tr '\n' ' ')"
done
for i in 1 2; do
  for l in libbase libpbccs_amd; do
    PBCCS_LIB=$GRAFT_REPO_ROOT/pbccs_amd/_lib/$l.so timeout -k 10 300 python -u bench.py --cpu-sample 0 > $OUT/p_${l}_$i.json 2> $OUT/p_${l}_$i.err || { echo "bench $l failed"; tail -20 $OUT/p_${l}_$i.err; exit 1; }
    echo "2kb $l: $(python -c "import json; d=json.load(open('$OUT/p_${l}_$i.json')); k=d['kernels']; print(d['value'], d['zmw_status'], {n: round(v['device_ms']/max(1,v['launches']),1) for n,v in k.items() if v['launches']})")"
  done
done
for sl in 2 4; do
  PBCCS_POA_SLICES=$sl timeout -k 10 300 python -u bench.py --stage ccs --steps 5 --warmup 1 --cpu-sample 0 > $OUT/ccs_s$sl.json 2> $OUT/ccs_s$sl.err || { echo "ccs $sl failed"; tail -20 $OUT/ccs_s$sl.err; exit 1; }
  echo "ccs slices $sl: $(python -c "import json; d=json.load(open('$OUT/ccs_s$sl.json')); print(d['value'], d['zmw_status'], d['poa_wall_ms'], d['poa_device_ms'], d['poa_thread_ms'])")"
done
for hr in 3200 1536; do
  PBCCS_HYBRID_ROWS=$hr timeout -k 10 400 python -u bench.py --workload 10kb --steps 8 --zmws-per-step 125 --warmup 0 --cpu-sample 0 > $OUT/b10_$hr.json 2> $OUT/b10_$hr.err || { echo "10kb $hr failed"; tail -20 $OUT/b10_$hr.err; exit 1; }
  echo "10kb x1000 hybrid rows $hr: $(python -c "import json; d=json.load(open('$OUT/b10_$hr.json')); print(d['value'], d['gcups'], d['zmw_status'], d['roofline']['in_flight'], d['band_memory_gb']['pool_mapped_bytes'])")"
done
