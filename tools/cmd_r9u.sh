# the whole GPU suite and smoke at the current sources
TAG=r9u bash tools/gpu_steps.sh tests && TAG=r9u bash tools/gpu_steps.sh smoke
