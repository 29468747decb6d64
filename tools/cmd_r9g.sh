TAG=r9g VARIANTS='PBCCS_SLOT_STREAMS=1 AMD_SERIALIZE_KERNEL=3 AMD_SERIALIZE_COPY=3;PBCCS_SLOT_STREAMS=1 AMD_SERIALIZE_COPY=3;PBCCS_SLOT_STREAMS=1 AMD_SERIALIZE_KERNEL=3' bash tools/oom_variants.sh && \
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k multiread -x -v --timeout 120 --timeout-method thread > gpurun_out/r9g/pytest_mt.log 2>&1; tail -3 gpurun_out/r9g/pytest_mt.log; \
TAG=r9g MIXN=1000 VARIANTS='PBCCS_HYBRID_LDS_KB=80 PBCCS_HYBRID_ROWS=4096;PBCCS_HYBRID_LDS_KB=150 PBCCS_HYBRID_ROWS=9216;NONE=1' bash tools/gpu_steps.sh abmixed && \
TAG=r9g ABSTEPS=6 ENVS="PBCCS_TALL_SCAN_PROBE=1 -" bash tools/gpu_steps.sh ab_env
