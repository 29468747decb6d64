# certified scan on the 16-lane fills: parity, then the headline A/B (PBCCS_SCAN_PATHS=5 vs the default 1)
mkdir -p gpurun_out/r9zc
timeout -k 10 900 python3 -u -m pytest tests/test_certified_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r9zc/pytest_cert.log 2>&1; rc=$?; tail -3 gpurun_out/r9zc/pytest_cert.log; [ $rc -eq 0 ] || exit $rc
TAG=r9zc ABSTEPS=10 ENVS="PBCCS_SCAN_PATHS=5 PBCCS_SCAN_PATHS=1" bash tools/gpu_steps.sh ab_env
for k in 1 2 3 4; do python3 -c "import json; d=json.load(open('gpurun_out/r9zc/ab_env_$k.json')); print(d['value'], d.get('certified_scan'))"; done
