# packed transfers: parity, then the ccs stage and the headline against the tree before them (_lib_ab)
mkdir -p gpurun_out/r9w
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_schedule.py tests/test_certified_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r9w/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r9w/pytest.log; [ $rc -eq 0 ] || exit $rc
TAG=r9w ABARGS="--stage ccs" bash tools/gpu_steps.sh ab_lib && TAG=r9w2 bash tools/gpu_steps.sh ab_lib
