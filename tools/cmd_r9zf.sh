# pinned staging retired instead of freed mid-run: configs[3] at 1000 ZMWs, interleaved against HEAD's engine (_lib_ab)
TAG=r9zf MIXN=1000 MIXARGS="--cpu-sample 0" VARIANTS="NONE=1;PBCCS_LIB=pbccs_amd/_lib_ab/libpbccs_amd.so;NONE=1;PBCCS_LIB=pbccs_amd/_lib_ab/libpbccs_amd.so" bash tools/gpu_steps.sh abmixed
