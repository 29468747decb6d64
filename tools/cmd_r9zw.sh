# final: the whole GPU suite, smoke, the driver's command
TAG=r9zw bash tools/gpu_steps.sh tests && TAG=r9zw bash tools/gpu_steps.sh smoke && TAG=r9zw bash tools/gpu_steps.sh bench
