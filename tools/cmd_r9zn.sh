# configs[3] at 2000 ZMWs: per-slot budget x0.85 vs default (the length-first order ran the device out of memory once)
TAG=r9zn MIXN=2000 MIXARGS="--cpu-sample 0" VARIANTS="NONE=1;PBCCS_QUEUE_BUDGET_SCALE=0.85;NONE=1;PBCCS_QUEUE_BUDGET_SCALE=0.85" bash tools/gpu_steps.sh abmixed
for k in 1 2 3 4; do python3 -c "import json; d=json.load(open('gpurun_out/r9zn/abmixed_$k.json')); print($k, d['value'], d['polished'], d['oom_retries'])"; done
