# configs[3] at 1000 ZMWs at the current sources: HIP API blocking and per-slot device gaps
TAG=r9ze MIXN=1000 bash tools/gpu_steps.sh apimixed > /dev/null && \
python3 tools/slot_gaps.py "$(find gpurun_out/r9ze/apimixed -name '*kernel_trace.csv' | head -1)" 1.0 > gpurun_out/r9ze/slot_gaps.json && \
python3 -c "
import json; d=json.load(open('gpurun_out/r9ze/api_gaps.json'))
for k,v in list(d['by_function'].items())[:8]: print(k, v)
g=json.load(open('gpurun_out/r9ze/slot_gaps.json')); print(g['span_s'], g['classes'], g['tall_waves'], g['slot_gap_total_s'])"
