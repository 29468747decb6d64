# round-6 evidence at the final kernel sources: PMC traffic, VALU per cell, wave-cycle decomposition, the
# occupancy line, the single-slot line, then the driver's command
TAG=r9z bash tools/gpu_steps.sh evidence
