# same-VA remap fix: the slot-stream OOM rerun (logged), then the OOM / pool-release GPU tests
TAG=r9t VARIANTS="PBCCS_SLOT_STREAMS=1 PBCCS_DBG_VA=1;PBCCS_DBG_VA=1" bash tools/oom_variants.sh || exit 1
for k in 1 2; do echo "== variant $k"; grep -E "vmpool|deferred|oom_retries|differing" gpurun_out/r9t/oom_$k.log | head -20; done
timeout -k 10 600 python3 -u -m pytest tests/test_schedule.py tests/test_poa_gpu.py -k "out_of_memory or pool_release" -x -v --timeout 300 --timeout-method thread > gpurun_out/r9t/pytest_oom.log 2>&1; rc=$?; tail -6 gpurun_out/r9t/pytest_oom.log; exit $rc
