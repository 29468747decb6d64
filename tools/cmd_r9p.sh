# headline wave-cycle decomposition (one PMC pass), then configs[3]: checkpoint interval / threshold (ZMWs in flight)
TAG=r9p bash tools/gpu_steps.sh binding || exit 1
TAG=r9p MIXN=1000 MIXARGS="--cpu-sample 0" VARIANTS="PBCCS_CKPT_K=8;PBCCS_CKPT_K=16;PBCCS_CKPT_K=32 PBCCS_CKPT_MIN_LEN=2000" bash tools/gpu_steps.sh abmixed
for k in 1 2 3; do python3 -c "import json; d=json.load(open('gpurun_out/r9p/abmixed_$k.json')); print(d['value'], d['polished'], d.get('oom_retries'), d.get('band_memory_gb'), {n: round(v['device_ms']/1e3,1) for n,v in d['kernels'].items()})"; done
