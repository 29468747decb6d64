# LDS-only tall fills with loads one chunk ahead: fill parity, then the headline A/B against -DPBCCS_TALL_PREFETCH=0
mkdir -p gpurun_out/r9r
timeout -k 10 900 python3 -u -m pytest tests/test_certified_gpu.py tests/test_gpu_parity.py -k "fill or certified or polish_batch" -x -v --timeout 300 --timeout-method thread > gpurun_out/r9r/pytest_fill.log 2>&1; rc=$?; tail -3 gpurun_out/r9r/pytest_fill.log; [ $rc -eq 0 ] || exit $rc
TAG=r9r bash tools/gpu_steps.sh ab_lib
