#!/bin/bash
# tools/oom_dbg.py (the out-of-memory rerun on a slot-shared stream, most of the device held) under each variant of
# VARIANTS (";"-separated "VAR=x VAR2=y" lists); one line per variant with the retries and the differing ZMWs.
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-oomvar}; mkdir -p $OUT; k=0
IFS=';' read -ra VS <<< "${VARIANTS:-NONE=1}"
for v in "${VS[@]}"; do
  k=$((k+1))
  ( eval "export $v"; timeout -k 10 240 python3 -u tools/oom_dbg.py ${OOM_LEAVE:-20} queue ) > $OUT/oom_$k.log 2>&1 || \
    { echo "variant $k failed"; tail -5 $OUT/oom_$k.log; exit 1; }
  echo "$v: $(grep -E 'oom_retries|differing' $OUT/oom_$k.log | tr '\n' ' ')"
done
