# rocprofv3 summary of the driver's command, the ccs stage line, configs[3] at 2000 ZMWs with its CPU leg
TAG=r9za bash tools/gpu_steps.sh prof && TAG=r9za bash tools/gpu_steps.sh ccs && TAG=r9za bash tools/gpu_steps.sh mixed
