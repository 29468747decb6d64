# ccs stage at 10 steps (20,000 ZMWs in one call): planned 2000-ZMW chunks vs 1000-ZMW chunks, interleaved
mkdir -p gpurun_out/r9zt
for rep in 1 2; do for c in 0 1000; do
  timeout -k 10 300 python3 -u bench.py --stage ccs --steps 10 --warmup 1 --cpu-sample 0 --ccs-chunk $c > gpurun_out/r9zt/ccs_${c}_$rep.json 2> gpurun_out/r9zt/ccs_${c}_$rep.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r9zt/ccs_${c}_$rep.json')); print('chunk $c', d['value'])"
done; done
