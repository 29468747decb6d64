# configs[3] at 2000 ZMWs: speculative band headroom leaving 48 GB free vs 24 (the length-first order's OOM reruns)
TAG=r9zp MIXN=2000 MIXARGS="--cpu-sample 0" VARIANTS="NONE=1;PBCCS_HEADROOM_MARGIN_GB=48;NONE=1;PBCCS_HEADROOM_MARGIN_GB=48" bash tools/gpu_steps.sh abmixed > /dev/null
for k in 1 2 3 4; do python3 -c "import json; d=json.load(open('gpurun_out/r9zp/abmixed_$k.json')); print($k, d['value'], d['polished'], d['oom_retries'])"; done
