# configs[3] at 1000 ZMWs: hybrid fills with loads one chunk ahead at one wave per SIMD (default) vs without at two
TAG=r9zr MIXN=1000 MIXARGS="--cpu-sample 0" VARIANTS="NONE=1;PBCCS_LIB=pbccs_amd/_lib_ab/libpbccs_amd.so;NONE=1;PBCCS_LIB=pbccs_amd/_lib_ab/libpbccs_amd.so" bash tools/gpu_steps.sh abmixed > /dev/null
for k in 1 2 3 4; do python3 -c "import json; d=json.load(open('gpurun_out/r9zr/abmixed_$k.json')); print($k, d['value'], d['polished']['zmws_per_s'], d['oom_retries'], round(d['kernels']['k_fill_tall']['device_ms']/1e3,1))"; done
