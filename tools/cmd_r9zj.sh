# batches ordered by template length first: configs[3] at 1000 ZMWs against HEAD's planner (_lib_ab), interleaved
TAG=r9zj MIXN=1000 MIXARGS="--cpu-sample 0" VARIANTS="NONE=1;PBCCS_LIB=pbccs_amd/_lib_ab/libpbccs_amd.so;NONE=1;PBCCS_LIB=pbccs_amd/_lib_ab/libpbccs_amd.so" bash tools/gpu_steps.sh abmixed
