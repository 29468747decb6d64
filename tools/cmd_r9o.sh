# hybrid fills with loads one chunk ahead: long-read parity, then configs[3] A/B of the scan paths
mkdir -p gpurun_out/r9o
timeout -k 10 900 python3 -u -m pytest tests/test_certified_gpu.py tests/test_ckpt_gpu.py "tests/test_gpu_parity.py::test_fills_10kb_match_oracle" "tests/test_gpu_parity.py::test_polish_10kb_batch_matches_oracle" "tests/test_gpu_parity.py::test_polish_mixed_long_matches_fixture" "tests/test_gpu_parity.py::test_polish_20kb_matches_fixture" -x -v --timeout 300 --timeout-method thread > gpurun_out/r9o/pytest_long.log 2>&1; rc=$?; tail -4 gpurun_out/r9o/pytest_long.log; [ $rc -eq 0 ] || exit $rc
TAG=r9o MIXN=1000 MIXARGS="--cpu-sample 0" VARIANTS="PBCCS_SCAN_PATHS=1;PBCCS_SCAN_PATHS=3" bash tools/gpu_steps.sh abmixed
for k in 1 2; do python3 -c "import json; d=json.load(open('gpurun_out/r9o/abmixed_$k.json')); print(d['value'], d['polished'], d.get('certified_scan'), d.get('oom_retries'), {n: round(v['device_ms']/1e3,1) for n,v in d['kernels'].items()})"; done
