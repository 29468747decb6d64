# final: the whole GPU suite, smoke, the driver's command
TAG=r9zx2 bash tools/gpu_steps.sh tests && TAG=r9zx2 bash tools/gpu_steps.sh smoke && TAG=r9zx2 bash tools/gpu_steps.sh bench
