# ccs stage HIP API trace: blocking calls by function and the long ones
TAG=r9zh bash tools/gpu_steps.sh apiccs > /dev/null && python3 tools/api_gaps.py "$(find gpurun_out/r9zh/apiccs -name '*hip_api_trace.csv' | head -1)" 50 > gpurun_out/r9zh/api_gaps.json && rm -f "$(find gpurun_out/r9zh/apiccs -name '*hip_api_trace.csv' | head -1)" && python3 -c "
import json; d=json.load(open('gpurun_out/r9zh/api_gaps.json'))
for k,v in list(d['by_function'].items())[:10]: print(k, v)
import collections; c=collections.Counter(x['fn'] for x in d['long_calls']); print(c, d['long_calls_total_s'])"
