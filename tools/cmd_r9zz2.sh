# unmapped ranges freed at once, reused reservations parked: memory across repetitions, the slot-stream OOM rerun
mkdir -p gpurun_out/r9zz2
PBCCS_DBG_VA=1 timeout -k 10 400 python3 -u -m pytest tests/test_schedule.py tests/test_poa_gpu.py -k "memory_does_not_grow or out_of_memory or pool_release" -x -v --timeout 300 --timeout-method thread > gpurun_out/r9zz2/p.log 2>&1; rc=$?; tail -3 gpurun_out/r9zz2/p.log; [ $rc -eq 0 ] || exit $rc
TAG=r9zz2 VARIANTS="PBCCS_SLOT_STREAMS=1 PBCCS_DBG_VA=1" bash tools/oom_variants.sh && grep -E "vmpool|differing" gpurun_out/r9zz2/oom_1.log | head -12
