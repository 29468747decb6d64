# certified tall fills scaling by a reciprocal: parity, then the headline A/B against the exact path
mkdir -p gpurun_out/r9zd
timeout -k 10 900 python3 -u -m pytest tests/test_certified_gpu.py tests/test_gpu_parity.py -k "certified or fill or polish_batch" -x -v --timeout 300 --timeout-method thread > gpurun_out/r9zd/pytest_cert.log 2>&1; rc=$?; tail -3 gpurun_out/r9zd/pytest_cert.log; [ $rc -eq 0 ] || exit $rc
TAG=r9zd ABSTEPS=10 ENVS="- PBCCS_CERTIFIED_SCAN=0" bash tools/gpu_steps.sh ab_env
for k in 1 2 3 4; do python3 -c "import json; d=json.load(open('gpurun_out/r9zd/ab_env_$k.json')); print(d['value'], d.get('certified_scan'))"; done
