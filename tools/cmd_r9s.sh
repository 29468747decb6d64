# the out-of-memory rerun on slot-shared streams, with every pool reservation / unmap logged (PBCCS_DBG_VA=1)
TAG=r9s VARIANTS="PBCCS_SLOT_STREAMS=1 PBCCS_DBG_VA=1;PBCCS_DBG_VA=1" bash tools/oom_variants.sh
for k in 1 2; do echo "== variant $k"; grep -E "vmpool|deferred|oom_retries|differing" gpurun_out/r9s/oom_$k.log | head -40; done
