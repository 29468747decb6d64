mkdir -p gpurun_out/r9m
timeout -k 10 900 python3 -u -m pytest tests/test_certified_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r9m/pytest_cert.log 2>&1; rc=$?; tail -4 gpurun_out/r9m/pytest_cert.log; [ $rc -eq 0 ] || exit $rc
TAG=r9m MIXN=1000 MIXARGS="--cpu-sample 0" VARIANTS="PBCCS_SCAN_PATHS=3;PBCCS_SCAN_PATHS=1;PBCCS_CERTIFIED_SCAN=0" bash tools/gpu_steps.sh abmixed
for k in 1 2 3; do python3 -c "import json; d=json.load(open('gpurun_out/r9m/abmixed_$k.json')); print(d['value'], d.get('certified_scan'), d.get('oom_retries'))"; done
