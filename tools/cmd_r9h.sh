TAG=r9h MIXN=1000 VARIANTS='PBCCS_QUEUE_BUDGET_SCALE=1.6;MIXSTREAMS=12 GPU_MAX_HW_QUEUES=32;NONE=1' bash tools/gpu_steps.sh abmixed && \
GPU_MAX_HW_QUEUES=32 TAG=r9h ARGV="--streams 8;--streams 12" bash tools/gpu_steps.sh ab_args
