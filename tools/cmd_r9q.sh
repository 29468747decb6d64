# configs[3]: where the fills' computed cells go (count-only regrow / overflow refills) at checkpoint interval 8 and 16
TAG=r9q MIXN=1000 MIXARGS="--cpu-sample 0" VARIANTS="PBCCS_FILL_WORK=1 PBCCS_CKPT_K=8;PBCCS_FILL_WORK=1 PBCCS_CKPT_K=16" bash tools/gpu_steps.sh abmixed
for k in 1 2; do python3 -c "import json; d=json.load(open('gpurun_out/r9q/abmixed_$k.json')); print(d['value'], json.dumps(d.get('fill_work')), {n: round(v['device_ms']/1e3,1) for n,v in d['kernels'].items()})"; done
