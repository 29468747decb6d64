mkdir -p gpurun_out/r9i
timeout -k 10 900 python3 -u -m pytest tests/test_certified_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r9i/pytest_cert.log 2>&1; rc=$?; tail -5 gpurun_out/r9i/pytest_cert.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_ckpt_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r9i/pytest_parity.log 2>&1; rc=$?; tail -3 gpurun_out/r9i/pytest_parity.log; [ $rc -eq 0 ] || exit $rc
TAG=r9i ABSTEPS=10 ENVS="- PBCCS_CERTIFIED_SCAN=0" bash tools/gpu_steps.sh ab_env
