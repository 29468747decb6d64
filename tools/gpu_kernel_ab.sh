#!/bin/bash
# GPU box: Arrow parity suite on the in-tree build, then interleaved profiled benches of two builds (PBCCS_LIB:
# pbccs_amd/_lib/libold.so vs libnew.so), printing one kernel's device time (KERNEL, default k_suffix).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-sab}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_schedule.py -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2; do
  for l in libold libnew; do
    PBCCS_LIB=$GRAFT_REPO_ROOT/pbccs_amd/_lib/$l.so timeout -k 10 300 python -u bench.py --cpu-sample 0 > $OUT/${l}_$i.json 2> $OUT/${l}_$i.err || { echo "bench $l failed"; tail -20 $OUT/${l}_$i.err; exit 1; }
    echo "$l: $(python -c "import json; d=json.load(open('$OUT/${l}_$i.json')); k=d['kernels']['${KERNEL:-k_suffix}']; print(d['value'], k['launches'], k['device_ms'])")"
  done
done
