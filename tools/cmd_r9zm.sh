# final configs[3] 2000-ZMW line and configs[4] two-rank rehearsal at 10,000 ZMWs
TAG=r9zm bash tools/gpu_steps.sh mixed && TAG=r9zm CELLTO=800 bash tools/gpu_steps.sh cell2
