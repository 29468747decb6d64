TAG=r9f VARIANTS='PBCCS_SLOT_STREAMS=1 PBCCS_DBG_JOINSYNC=1;PBCCS_SLOT_STREAMS=1;NONE=1' bash tools/oom_variants.sh && \
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k multiread -x -v --timeout 120 --timeout-method thread > gpurun_out/r9f/pytest_mt.log 2>&1; tail -3 gpurun_out/r9f/pytest_mt.log; \
TAG=r9f MIXN=1000 VARIANTS='NONE=1;PBCCS_D2H_DRAIN=0;PBCCS_TALL_SCAN_PROBE=1' bash tools/gpu_steps.sh abmixed
