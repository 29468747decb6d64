# configs[3] at 1000 ZMWs: hybrid LDS budget 40 KB per read and checkpoint interval 16 against the defaults, interleaved
TAG=r9zi MIXN=1000 MIXARGS="--cpu-sample 0" VARIANTS="NONE=1;PBCCS_HYBRID_LDS_KB=40;PBCCS_CKPT_K=16;NONE=1;PBCCS_HYBRID_LDS_KB=40;PBCCS_CKPT_K=16" bash tools/gpu_steps.sh abmixed
