#!/bin/bash
# GPU box: final evidence part 1 at the working tree, then the Quiver stage A/B of the host-side parallel loops
# and page-locked read pools (working tree) against HEAD (libbase.so).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TAG=f1 bash tools/gpu_final1.sh || exit 1
OUT=gpurun_out/r3w
mkdir -p $OUT
run() {   # name, env...
  local name=$1; shift
  env "$@" PBCCS_QUIVER_TRACE=1 timeout -k 10 240 python -u bench.py --stage quiver --steps 5 --warmup 1 --cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -20 $OUT/$name.err; return 1; }
  echo "$name: $(python -c "import json; d=json.load(open('$OUT/$name.json')); print(d['value'], d['ms_per_step'])")"
}
run new && run base PBCCS_LIB=$PWD/pbccs_amd/_lib/libbase.so && run new2 && run base2 PBCCS_LIB=$PWD/pbccs_amd/_lib/libbase.so && \
grep '\[quiver\]' $OUT/new2.err | tail -9
