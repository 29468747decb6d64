# ccs chunks sized by the call: the ccs GPU tests, then the stage line at round 5's shape (twice) and at 10 steps
mkdir -p gpurun_out/r9zu
timeout -k 10 600 python3 -u -m pytest tests/test_poa_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r9zu/pytest_poa.log 2>&1; rc=$?; tail -2 gpurun_out/r9zu/pytest_poa.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do timeout -k 10 300 python3 -u bench.py --stage ccs --steps 5 --warmup 1 > gpurun_out/r9zu/ccs5_$r.json 2> gpurun_out/r9zu/ccs5_$r.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r9zu/ccs5_$r.json')); print('5 steps', d['value'], d['parity_sample']['ok'])"; done
timeout -k 10 300 python3 -u bench.py --stage ccs --steps 10 --warmup 2 > gpurun_out/r9zu/ccs10.json 2> gpurun_out/r9zu/ccs10.err && python3 -c "import json; d=json.load(open('gpurun_out/r9zu/ccs10.json')); print('10 steps', d['value'], d['parity_sample']['ok'])"
