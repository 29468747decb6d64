# ccs chunks sized by the call (~10 per call, 1000-2000 ZMWs) vs HEAD's 2000 (_lib_ab): 5 steps, interleaved
mkdir -p gpurun_out/r9zv
for rep in 1 2; do for L in pbccs_amd/_lib/libpbccs_amd.so pbccs_amd/_lib_ab/libpbccs_amd.so; do
  PBCCS_LIB=$L timeout -k 10 300 python3 -u bench.py --stage ccs --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/r9zv/c.json 2> gpurun_out/r9zv/c.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r9zv/c.json')); print('$L', d['value'])"
done; done
