#!/bin/bash
# Host side (build container): run one gpurun call; call it again (at most 3 more times) only when gpurun
# reports an infrastructure-transient status -- the box was lost before the command ran, nothing executed and
# nothing was charged.  Any other outcome (pass, fail, timeout) is final.  Usage: tools/gpurun_retry.sh LOG TIMEOUT CMD
LOG=$1; TO=$2; shift 2
for i in $(seq 1 ${RETRIES:-4}); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  grep -q "status=transient\|backing off" "$LOG" || break
  echo "[retry $i: transient]" >> "$LOG.retries"
  # a back-off names its wait ("retry in Ns"): sleep that long (plus a margin), else 45 s
  W=$(grep -o "retry in [0-9]*s" "$LOG" | tail -1 | grep -o "[0-9]*")
  sleep $(( ${W:-30} + 15 ))
done
echo done >> "$LOG"
