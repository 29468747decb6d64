# configs[3] at 1000 ZMWs: 8 vs 12 workspace slots, interleaved
for rep in 1 2; do for s in 8 12; do
  TAG=r9zl_${s}_$rep MIXN=1000 MIXSTREAMS=$s MIXARGS="--cpu-sample 0" bash tools/gpu_steps.sh abmixed | tail -1 | cut -c1-120 || exit 1
done; done
